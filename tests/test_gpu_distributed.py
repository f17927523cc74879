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
