"""GPU: the sharded servers with the real HIP kernels, 2 ranks, two rounds each.

``gloo``: both ranks on one GPU (the single-GPU test box).  ``nccl`` (RCCL over
xGMI): one GPU per rank, run where two GPUs are visible and skipped otherwise;
the collectives are the same calls.  Every round's broadcast must be retired by
the rank's local workers (no round result left in the queue).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests import golden as G

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, backend, outq):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(rank if backend == "nccl" else 0)
    dist.init_process_group(backend, rank=rank, world_size=world)
    from distributed_learning_simulator_amd.distributed import (ShardedFedQuantServer,
                                                                ShardedFedServer,
                                                                ShardedSignSGDServer)
    out = {}
    # FedAvg
    z = G.load("fedavg.npz")
    case = G.meta(z)[1]
    k, layout, K = case["key"], case["layout"], case["K"]
    U, n = z[f"{k}_U"], z[f"{k}_n"]
    s = ShardedFedServer(tester=None, worker_number=K, synchronous=True)
    q = s.worker_data_queue
    for w in s.local_worker_ids:  # the initial broadcast
        q.get_result(consumer=w, timeout=60)
    fed = []
    for _round in range(2):
        for wid in s.local_worker_ids:
            d = {nm: torch.from_numpy(v.copy()) for nm, v in G.split(U[wid], layout).items()}
            q.add_task((wid, int(n[wid]), d))
        for w in s.local_worker_ids:
            res = q.get_result(consumer=w, timeout=60)
        assert len(q._results) == 0, "round result left in the queue"
        fed.append(np.concatenate([res[nm].reshape(-1).cpu().numpy() for nm, _ in layout]))
    assert np.array_equal(fed[0].view(np.uint32), fed[1].view(np.uint32))
    out["fed"] = fed[0]
    # bit-exact exchange (parameter slices, all-to-all + all-gather)
    sx = ShardedFedServer(tester=None, worker_number=K, synchronous=True, exchange="alltoall",
                          order="worker_id")
    qx = sx.worker_data_queue
    for w in sx.local_worker_ids:
        qx.get_result(consumer=w, timeout=60)
    for wid in reversed(sx.local_worker_ids):
        d = {nm: torch.from_numpy(v.copy()) for nm, v in G.split(U[wid], layout).items()}
        qx.add_task((wid, int(n[wid]), d))
    for w in sx.local_worker_ids:
        res = qx.get_result(consumer=w, timeout=60)
    assert len(qx._results) == 0
    out["fed_exact"] = np.concatenate([res[nm].reshape(-1).cpu().numpy() for nm, _ in layout])
    # sign vote
    zs = G.load("sign_vote.npz")
    cs = G.meta(zs)[1]
    S = zs["c1_signs"]
    ss = ShardedSignSGDServer(tester=None, worker_number=cs["K"], synchronous=True)
    for wid in ss.local_worker_ids:
        ss.worker_data_queue.add_task(
            [torch.from_numpy(v.copy()) for v in G.split(S[wid], cs["layout"]).values()])
    res = ss.worker_data_queue.get_result(consumer=0, timeout=60)
    out["sign"] = np.concatenate([t.reshape(-1).cpu().numpy() for t in res])
    # fed_quant
    zq = G.load("dequant.npz")
    cq = G.meta(zq)[0]
    sq = ShardedFedQuantServer(tester=None, worker_number=cq["K"], synchronous=True)
    qq = sq.worker_data_queue
    for w in sq.local_worker_ids:  # the initial broadcast
        qq.get_result(consumer=w, timeout=60)
    for _round in range(2):
        for i in sq.local_worker_ids:
            d = {}
            for name, shape in cq["layout"]:
                if name in cq["qnames"]:
                    d[name] = tuple(torch.from_numpy(zq[f"q{i}_{name}_{x}"].copy())
                                    for x in ("int", "scale", "zp"))
                else:
                    d[name] = torch.from_numpy(zq[f"q{i}_{name}_f32"].copy())
            qq.add_task((i, int(zq["n"][i]), d))
        for w in sq.local_worker_ids:
            qq.get_result(consumer=w, timeout=60)
        assert len(qq._results) == 0, "fed_quant round result left in the queue"
    agg = sq.last_aggregate
    out["quant"] = np.concatenate([agg[nm].reshape(-1).cpu().numpy() for nm, _ in cq["layout"]])
    # the column-chunked pipeline (3 chunks, the default) against one chunk, in both
    # aggregation modes: the same per-tile kernels and partial sums (a + b == b + a)
    for mode in ("exact", "fma"):
        got = {}
        for chunks in (3, 1):
            sc = ShardedFedQuantServer(tester=None, worker_number=cq["K"], synchronous=True,
                                       chunks=chunks, aggregation_mode=mode)
            qc = sc.worker_data_queue
            for w in sc.local_worker_ids:
                qc.get_result(consumer=w, timeout=60)
            for i in sc.local_worker_ids:
                d = {}
                for name, shape in cq["layout"]:
                    if name in cq["qnames"]:
                        d[name] = tuple(torch.from_numpy(zq[f"q{i}_{name}_{x}"].copy())
                                        for x in ("int", "scale", "zp"))
                    else:
                        d[name] = torch.from_numpy(zq[f"q{i}_{name}_f32"].copy())
                qc.add_task((i, int(zq["n"][i]), d))
            for w in sc.local_worker_ids:
                qc.get_result(consumer=w, timeout=60)
            a = sc.last_aggregate
            got[chunks] = np.concatenate([a[nm].reshape(-1).cpu().numpy()
                                          for nm, _ in cq["layout"]])
        out[f"quant_{mode}_chunked"] = got[3]
        out[f"quant_{mode}_whole"] = got[1]
    outq.put((rank, out))
    dist.destroy_process_group()


@pytest.mark.parametrize("backend", ["gloo", "nccl"])
def test_sharded_servers_two_ranks(backend):
    if backend == "nccl" and torch.cuda.device_count() < 2:
        pytest.skip("RCCL needs one GPU per rank")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, backend, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = dict(q.get(timeout=170) for _ in range(2))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    z = G.load("fedavg.npz")
    k = G.meta(z)[1]["key"]
    ref = z[f"{k}_full"]
    for r in (0, 1):
        got = outs[r]["fed"]
        assert np.linalg.norm(got - ref) / np.linalg.norm(ref) < 1e-6
        assert np.array_equal(outs[r]["sign"].view(np.uint32),
                              G.load("sign_vote.npz")["c1_vote"].view(np.uint32))
        zq = G.load("dequant.npz")
        assert np.linalg.norm(outs[r]["quant"] - zq["agg"]) / np.linalg.norm(zq["agg"]) < 1e-6
    assert np.array_equal(outs[0]["fed"].view(np.uint32), outs[1]["fed"].view(np.uint32))
    # exchange="alltoall": bits of one server aggregating every client in worker-id order
    from oracle import _c
    case = G.meta(z)[1]
    ref = _c.fedavg_ref(z[f"{k}_U"], [int(x) for x in z[f"{k}_n"]], list(range(case["K"])))
    for r in (0, 1):
        assert np.array_equal(outs[r]["fed_exact"][: ref.size].view(np.uint32), ref.view(np.uint32))
        for mode in ("exact", "fma"):  # chunked == unchunked, bit for bit
            a, b = outs[r][f"quant_{mode}_chunked"], outs[r][f"quant_{mode}_whole"]
            assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), mode
            assert np.linalg.norm(a - zq["agg"]) / np.linalg.norm(zq["agg"]) < 1e-6, mode


def _shapley_worker(rank, world, port, tag, metric_dir, outq):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from distributed_learning_simulator_amd.distributed import (
        ShardedGTGShapleyValueServer, ShardedMultiRoundShapleyValueServer)
    from tests.test_gpu_shapley import _setup
    case = next(c for c in G.shapley_large_cases() if c["tag"] == tag)
    if tag.startswith("gtg"):
        server, layout, U = _setup(case, ShardedGTGShapleyValueServer)
    else:
        server, layout, U = _setup(case, ShardedMultiRoundShapleyValueServer,
                                   metric_dir=metric_dir)
    np.random.seed(case["seed"])
    local = server.local_worker_ids
    for w in local:  # the initial broadcast
        server.worker_data_queue.get_result(consumer=w, timeout=120)
    for i in local:  # a rank receives only its own clients
        d = {nm: torch.from_numpy(v.copy()) for nm, v in G.split(U[i], layout).items()}
        server.worker_data_queue.add_task((i, int(case["n"][i]), d))
    for w in local:
        server.worker_data_queue.get_result(consumer=w, timeout=300)
    assert server.parameters.store.U.is_cuda  # the HIP kernels, on the GPU
    sv = {int(k): float(v) for k, v in server.shapley_values[1].items()}
    outq.put((rank, sv, [tuple(x) for x in server.evaluated_subsets]))
    dist.destroy_process_group()


@pytest.mark.parametrize("tag", ["gtg_50_4", "multiround_12"])
def test_sharded_shapley_servers_two_ranks(tag, tmp_path):
    """the sharded Shapley servers with the HIP kernels on the
    GPU (gloo, 2 ranks on one GPU): each rank receives its own clients into its
    block of the store, the in-place all-gather fills the other block, the
    coalitions are dealt over the ranks and the utilities all-reduced.  Shapley
    values within 1e-12 of the reference's golden (BASELINE config 5 client
    counts), the union of the ranks' evaluated coalitions is the golden set (each
    evaluated once), and multiround's rank 0 writes the reference's metric_1 bytes."""
    case = next(c for c in G.shapley_large_cases() if c["tag"] == tag)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    dirs = [tmp_path / f"r{r}" for r in range(2)]
    for d in dirs:
        d.mkdir()
    procs = [ctx.Process(target=_shapley_worker, args=(r, 2, port, tag, str(dirs[r]), q))
             for r in range(2)]
    for p in procs:
        p.start()
    outs = dict((r, (sv, ev)) for r, sv, ev in _collect(procs, q, 2, 200))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for r in (0, 1):
        sv = outs[r][0]
        for k, v in case["sv"].items():
            assert abs(sv[int(k)] - v) <= 1e-12, (tag, r, k)
    ev0, ev1 = outs[0][1], outs[1][1]
    assert not set(ev0) & set(ev1)  # dealt, not duplicated
    assert len(ev0) + len(ev1) == case["n_evaluated"]
    assert set(ev0) | set(ev1) == set(case["evaluated"])
    if case["metric_pickle"] is not None:  # rank 0 writes the metric_<round> side file
        assert (dirs[0] / "metric_1").read_bytes() == case["metric_pickle"]
        assert not (dirs[1] / "metric_1").exists()


def _collect(procs, q, n, timeout):
    """n results from the queue; fails as soon as a process exits without one
    (a child's exception would otherwise leave the parent waiting out the timeout)."""
    import queue as _queue
    import time as _time
    out, t0 = [], _time.monotonic()
    while len(out) < n:
        try:
            out.append(q.get(timeout=2))
            continue
        except _queue.Empty:
            pass
        dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
        assert not dead, f"a worker process failed: exit codes {dead}"
        assert _time.monotonic() - t0 < timeout, "workers timed out"
    return out


def _logits_worker(seed, outq):
    torch.cuda.set_device(0)
    from distributed_learning_simulator_amd.models import ResNet18, synthetic_classification
    from distributed_learning_simulator_amd.trainer import Inferencer
    torch.manual_seed(seed)
    model = ResNet18().to("cuda:0")
    X, y = synthetic_classification(10000, (3, 32, 32), seed=11)
    inf = Inferencer(model, (X, y), device=torch.device("cuda", 0))
    lg = inf.logits()
    loss, acc, _ = inf.inference()
    outq.put((lg.cpu().numpy(), float(loss), acc))


def test_utility_bit_identical_across_processes():
    """the multi-rank GTG needs a coalition's utility to be the
    same on every rank.  Two fresh spawned processes (their own MIOpen algorithm
    choice, their own caches) evaluate the same ResNet-18 state on the same 10k
    images with the default Inferencer: bit-identical logits, equal loss and
    accuracy."""
    ctx = mp.get_context("spawn")
    res = []
    for _ in range(2):  # one after the other: each process alone on the GPU
        q = ctx.Queue()
        p = ctx.Process(target=_logits_worker, args=(7, q))
        p.start()
        res.extend(_collect([p], q, 1, 200))
        p.join(60)
        assert p.exitcode == 0
    (la, loss_a, acc_a), (lb, loss_b, acc_b) = res
    assert la.shape == (10000, 10)
    assert np.array_equal(la.view(np.uint32), lb.view(np.uint32))
    assert loss_a == loss_b and acc_a == acc_b
