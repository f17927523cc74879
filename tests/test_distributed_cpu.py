"""Multi-rank ``gloo`` tests (2, 3 and 8 ranks) of the sharded (multi-GPU) servers' host logic on CPU.

Kernels are replaced by numpy doubles (tests/cpu_doubles.py); what is tested is
the sharding (worker_id % world), the global sample count, the chunked
all-reduce, the int32 vote-count reduction and the Shapley utility fan-out.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests import golden as G

pytestmark = pytest.mark.slow


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tests import cpu_doubles
    cpu_doubles.install_global()


def _fedavg_worker(rank, world, port, outq):
    _init(rank, world, port)
    from distributed_learning_simulator_amd.distributed import ShardedFedServer
    z = G.load("fedavg.npz")
    case = G.meta(z)[1]
    k, layout, K = case["key"], case["layout"], case["K"]
    U, n = z[f"{k}_U"], z[f"{k}_n"]
    server = ShardedFedServer(tester=None, worker_number=K, synchronous=True,
                              device=torch.device("cpu"), chunks=3)
    q = server.worker_data_queue
    local = server.local_worker_ids
    for w in local:  # the initial broadcast, once per local worker
        q.get_result(consumer=w, timeout=30)
    assert len(q._results) == 0
    flats = []
    for _round in range(3):  # every round's broadcast is retired once each local worker took it
        for wid in local:
            d = {nm: torch.from_numpy(v.copy()) for nm, v in G.split(U[wid], layout).items()}
            q.add_task((wid, int(n[wid]), d))
        # a rank stores only its own clients' rows, not the global K
        assert server.parameters.store.capacity == len(local)
        for w in local:
            res = q.get_result(consumer=w, timeout=30)
        assert len(q._results) == 0, "round result left in the queue"
        flats.append(np.concatenate([res[nm].reshape(-1).numpy() for nm, _ in layout]))
    assert all(np.array_equal(f.view(np.uint32), flats[0].view(np.uint32)) for f in flats)
    outq.put((rank, local, flats[0]))
    dist.destroy_process_group()


def _fedavg_bitexact_worker(rank, world, port, outq):
    _init(rank, world, port)
    from distributed_learning_simulator_amd.distributed import ShardedFedServer
    z = G.load("fedavg.npz")
    case = G.meta(z)[1]
    k, layout, K = case["key"], case["layout"], case["K"]
    U, n = z[f"{k}_U"], z[f"{k}_n"]
    server = ShardedFedServer(tester=None, worker_number=K, synchronous=True,
                              device=torch.device("cpu"), exchange="alltoall", order="worker_id")
    q = server.worker_data_queue
    for w in server.local_worker_ids:
        q.get_result(consumer=w, timeout=30)
    for wid in reversed(server.local_worker_ids):  # order="worker_id": arrivals do not matter
        d = {nm: torch.from_numpy(v.copy()) for nm, v in G.split(U[wid], layout).items()}
        q.add_task((wid, int(n[wid]), d))
    for w in server.local_worker_ids:
        res = q.get_result(consumer=w, timeout=30)
    assert len(q._results) == 0
    outq.put((rank, np.concatenate([res[nm].reshape(-1).numpy() for nm, _ in layout])))
    dist.destroy_process_group()


def _fedavg_arrival_worker(rank, world, port, outq):
    """order="arrival": clients report in a fixed global sequence; the server's
    arrival clock is replaced by the client's position in it (the ranks' queue
    threads would otherwise stamp the node-wide monotonic clock), so the merged
    order must be that sequence — the order one reference server would have seen."""
    _init(rank, world, port)
    from distributed_learning_simulator_amd.distributed import ShardedFedServer
    z = G.load("fedavg.npz")
    case = G.meta(z)[1]
    k, layout, K = case["key"], case["layout"], case["K"]
    U, n = z[f"{k}_U"], z[f"{k}_n"]
    server = ShardedFedServer(tester=None, worker_number=K, synchronous=True,
                              device=torch.device("cpu"), exchange="alltoall")
    q = server.worker_data_queue
    for w in server.local_worker_ids:
        q.get_result(consumer=w, timeout=30)
    seq = np.random.RandomState(7).permutation(K).tolist()
    for rnd in range(2):  # the second round re-stamps every arrival
        order = seq if rnd == 0 else seq[::-1]
        for t, wid in enumerate(order):
            if wid in server.local_worker_ids:
                server._clock = lambda t=t: 1000 * rnd + t
                d = {nm: torch.from_numpy(v.copy()) for nm, v in G.split(U[wid], layout).items()}
                q.add_task((wid, int(n[wid]), d))
        for w in server.local_worker_ids:
            res = q.get_result(consumer=w, timeout=30)
        outq.put((rank, rnd, order, np.concatenate([res[nm].reshape(-1).numpy()
                                                     for nm, _ in layout])))
    dist.destroy_process_group()


def _sign_worker(rank, world, port, outq):
    _init(rank, world, port)
    from distributed_learning_simulator_amd.distributed import ShardedSignSGDServer
    z = G.load("sign_vote.npz")
    case = G.meta(z)[1]
    S, layout, K = z["c1_signs"], case["layout"], case["K"]
    server = ShardedSignSGDServer(tester=None, worker_number=K, synchronous=True,
                                  device=torch.device("cpu"))
    for wid in server.local_worker_ids:
        server.worker_data_queue.add_task(
            [torch.from_numpy(v.copy()) for v in G.split(S[wid], layout).values()])
    res = server.worker_data_queue.get_result(consumer=0, timeout=30)
    outq.put((rank, np.concatenate([t.reshape(-1).numpy() for t in res])))
    dist.destroy_process_group()


def _shapley_worker(rank, world, port, outq):
    _init(rank, world, port)
    from distributed_learning_simulator_amd.servers.GTG_shapley_value_server import \
        GTGShapleyValueServer
    case = next(c for c in G.shapley_cases() if c["tag"] == "gtg_5_2")
    layout = [(nm, tuple(s)) for nm, s in case["layout"]]
    K = case["K"]
    U = np.array(case["U"], np.float32)
    target = np.array(case["target"], np.float64)
    server = GTGShapleyValueServer(tester=None, worker_number=K, synchronous=True,
                                   device=torch.device("cpu"))
    server._set_prev_model(G.split(torch.tensor(case["prev"]), layout))

    def util(model, metric_type="acc"):
        v = np.concatenate([np.asarray(model[nm], np.float64).reshape(-1) for nm, _ in layout])
        d = v - target
        return float(1.0 / (1.0 + float(np.dot(d, d)) / case["scale"]))

    server.get_metric = util
    np.random.seed(case["seed"])
    for i in range(K):  # Shapley: every rank holds every client, evaluations fan out
        d = {nm: torch.from_numpy(v.copy()) for nm, v in G.split(U[i], layout).items()}
        server.worker_data_queue.add_task((i, int(case["n"][i]), d))
    outq.put((rank, {int(k): float(v) for k, v in server.shapley_values[1].items()},
              len(server.evaluated_subsets)))
    dist.destroy_process_group()


def _quant_payloads(K):
    """Synthetic fed_quant client payloads (ref servers/fed_quant_server.py:26-32):
    per-channel int8 / uint8 tensors with their (scale, zero point) and fp32 ones,
    sized so that the store's column chunks split tensors and tiles."""
    rng = np.random.RandomState(11)
    shapes = [("conv.weight", (16, 8, 3, 3), 1), ("conv.bias", (16,), 0),
              ("fc.weight", (24, 600), 1), ("fc.bias", (24,), 0), ("u8.weight", (20, 50), 2)]
    out = []
    for _ in range(K):
        d = {}
        for name, shape, kind in shapes:
            if kind == 0:
                d[name] = torch.from_numpy(rng.standard_normal(shape).astype(np.float32))
                continue
            lo, hi = (-128, 128) if kind == 1 else (0, 256)
            q = rng.randint(lo, hi, size=shape).astype(np.int8 if kind == 1 else np.uint8)
            sc = rng.uniform(1e-3, 1e-2, size=shape[0])
            zp = np.zeros(shape[0], np.int64) if kind == 1 else rng.randint(100, 150, shape[0])
            d[name] = (torch.from_numpy(q), torch.from_numpy(sc), torch.from_numpy(zp))
        out.append(d)
    return shapes, out


def _fed_quant_worker(rank, world, port, outq):
    _init(rank, world, port)
    from distributed_learning_simulator_amd.distributed import ShardedFedQuantServer
    K = 6
    shapes, payloads = _quant_payloads(K)
    res = {}
    for chunks in (3, 1):
        server = ShardedFedQuantServer(tester=None, worker_number=K, synchronous=True,
                                       device=torch.device("cpu"), chunks=chunks)
        q = server.worker_data_queue
        for w in server.local_worker_ids:
            q.get_result(consumer=w, timeout=30)
        for wid in server.local_worker_ids:
            q.add_task((wid, 10 + 3 * wid, payloads[wid]))
        for w in server.local_worker_ids:
            q.get_result(consumer=w, timeout=30)
        agg = server.last_aggregate
        res[chunks] = np.concatenate([agg[nm].reshape(-1).numpy() for nm, _, _ in shapes])
        if chunks == 3:  # the pipelined path really ran in 3 column ranges
            assert len(server.parameters.store._col_tables) == 3
    outq.put((rank, res[3], res[1]))
    dist.destroy_process_group()


def _spawn(fn, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=fn, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    return sorted(out, key=lambda x: x[0])


def test_sharded_fedavg_two_ranks():
    z = G.load("fedavg.npz")
    case = G.meta(z)[1]
    k = case["key"]
    out = _spawn(_fedavg_worker)
    assert out[0][1] == list(range(0, case["K"], 2)) and out[1][1] == list(range(1, case["K"], 2))
    assert np.array_equal(out[0][2].view(np.uint32), out[1][2].view(np.uint32))  # ranks agree
    from oracle.fedavg import fedavg_weighted
    ex = fedavg_weighted(z[f"{k}_U"], z[f"{k}_n"], range(case["K"]))
    got = out[0][2]
    assert np.linalg.norm(got - ex) / np.linalg.norm(ex) < 1e-6
    ref = z[f"{k}_full"]  # single-process reference result: same within normwise 1e-6
    assert np.linalg.norm(got - ref) / np.linalg.norm(ref) < 1e-6


@pytest.mark.parametrize("world", [2, 3, 8])
def test_sharded_fedavg_alltoall_bit_exact(world):
    """exchange="alltoall": bits identical to one server aggregating all K clients
    in worker-id order, for any number of ranks (8: the node the driver scales to)."""
    z = G.load("fedavg.npz")
    case = G.meta(z)[1]
    k = case["key"]
    out = _spawn(_fedavg_bitexact_worker, world)
    from oracle import _c
    U = z[f"{k}_U"]
    ref = _c.fedavg_ref(U, [int(x) for x in z[f"{k}_n"]], list(range(case["K"])))
    P = ref.size
    for _, got in out:
        assert np.array_equal(got[:P].view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_fedavg_alltoall_arrival_order(world):
    """exchange="alltoall", order="arrival": bits identical to one server summing
    the clients in the order they arrived over all ranks (ref
    servers/fed_server.py:69-73,81: self.parameters.keys() in insertion order)."""
    z = G.load("fedavg.npz")
    case = G.meta(z)[1]
    k = case["key"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fedavg_arrival_worker, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(2 * world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    from oracle import _c
    U = z[f"{k}_U"]
    ns = [int(x) for x in z[f"{k}_n"]]
    for _, _, order, got in out:
        ref = _c.fedavg_ref(U, ns, order)
        assert np.array_equal(got[:ref.size].view(np.uint32), ref.view(np.uint32))
    # the two rounds' orders give different bits (the order is really followed)
    r0 = next(g for _, rnd, _, g in out if rnd == 0)
    r1 = next(g for _, rnd, _, g in out if rnd == 1)
    assert not np.array_equal(r0.view(np.uint32), r1.view(np.uint32))


@pytest.mark.parametrize("world", [2, 8])
def test_sharded_sign_vote_bit_exact(world):
    z = G.load("sign_vote.npz")
    out = _spawn(_sign_worker, world)
    for _, v in out:
        assert np.array_equal(v.view(np.uint32), z["c1_vote"].view(np.uint32))


def test_shapley_fanout_two_ranks():
    case = next(c for c in G.shapley_cases() if c["tag"] == "gtg_5_2")
    out = _spawn(_shapley_worker)
    for _, sv, _n in out:
        for k, v in case["sv"].items():
            assert abs(sv[int(k)] - v) <= 1e-12
    assert out[0][2] + out[1][2] == len(case["evaluated"])  # the evaluations were split


def _sharded_gtg_worker(rank, world, port, outq):
    _init(rank, world, port)
    from distributed_learning_simulator_amd import factory
    case = next(c for c in G.shapley_cases() if c["tag"] == "gtg_6_3")
    layout = [(nm, tuple(s)) for nm, s in case["layout"]]
    K = case["K"]
    U = np.array(case["U"], np.float32)
    target = np.array(case["target"], np.float64)
    server = factory.get_server("GTG_shapley_value", tester=None, worker_number=K,
                                synchronous=True, device=torch.device("cpu"))
    assert type(server).__name__ == "ShardedGTGShapleyValueServer"
    server._set_prev_model(G.split(torch.tensor(case["prev"]), layout))

    def util(model, metric_type="acc"):
        v = np.concatenate([np.asarray(model[nm], np.float64).reshape(-1) for nm, _ in layout])
        d = v - target
        return float(1.0 / (1.0 + float(np.dot(d, d)) / case["scale"]))

    server.get_metric = util
    np.random.seed(case["seed"])
    for i in server.local_worker_ids:  # each rank only receives its own clients
        d = {nm: torch.from_numpy(v.copy()) for nm, v in G.split(U[i], layout).items()}
        server.worker_data_queue.add_task((i, int(case["n"][i]), d))
    outq.put((rank, {int(k): float(v) for k, v in server.shapley_values[1].items()}, 0))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_gtg_clients_sharded(world):
    """Each rank receives its own clients into its block of the store; one in-place
    all-gather fills the other blocks and the rows are adopted without a copy."""
    case = next(c for c in G.shapley_cases() if c["tag"] == "gtg_6_3")
    out = _spawn(_sharded_gtg_worker, world)
    for _, sv, _n in out:
        for k, v in case["sv"].items():
            assert abs(sv[int(k)] - v) <= 1e-12


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_fed_quant_chunked_pipeline(world):
    """ShardedFedQuantServer reduces its clients column chunk by column chunk (tile
    sub-tables) while the previous chunk's all-reduce is on the wire: the bits
    equal the unchunked sharded result, every rank agrees, and the aggregate is the
    dequant-then-FedAvg of all clients within the north-star 1e-6."""
    out = _spawn(_fed_quant_worker, world)
    for _, chunked, whole in out:
        assert np.array_equal(chunked.view(np.uint32), out[0][1].view(np.uint32))  # ranks agree
        if world == 2:  # a + b == b + a: the per-tile partials and their sum are the same bits
            assert np.array_equal(chunked.view(np.uint32), whole.view(np.uint32))
        else:  # 3 partials: the collective's summation order depends on the message size
            assert np.linalg.norm(chunked - whole) <= 1e-7 * np.linalg.norm(whole)
    from oracle.quant import dequant_fedavg
    K = 6
    shapes, payloads = _quant_payloads(K)
    clients = [{nm: (tuple(x.numpy() for x in v) if isinstance(v, tuple) else v.numpy())
                for nm, v in p.items()} for p in payloads]
    ref = dequant_fedavg(clients, [10 + 3 * w for w in range(K)], list(range(K)),
                         [(nm, shape) for nm, shape, _ in shapes])
    got = out[0][1]
    assert np.linalg.norm(got - ref) / np.linalg.norm(ref) < 1e-6


def test_queued_evaluations_match_get_metric(monkeypatch):
    """ShapleyValueServer.evaluate_subsets queues the default accuracy metric on a
    tester with correct_async (one host synchronisation per batch) and gives the
    floats get_metric gives; a get_metric replaced on the instance is honoured."""
    import torch
    from distributed_learning_simulator_amd.servers.fed_server import FedServer
    from distributed_learning_simulator_amd.servers.shapley_value_server import ShapleyValueServer

    class _Tester:
        def __init__(self):
            self.model = torch.nn.Linear(2, 1)
            self.dataset = (torch.zeros(7, 2), torch.zeros(7, dtype=torch.long))
            self.calls = []

        def count(self):
            return int(round(float(self.model.weight.detach().sum()))) % 8

        def correct_async(self):
            self.calls.append("async")
            return torch.tensor(self.count())

        def inference(self):
            self.calls.append("sync")
            self.accuracy_metric.value = self.count() / 7

    class _Acc:
        value = None

        def get_accuracy(self, _epoch=1):
            return self.value

    class _Params(dict):
        store = None

    from tests import cpu_doubles
    cpu_doubles.install(monkeypatch)
    tester = _Tester()
    tester.accuracy_metric = _Acc()
    server = ShapleyValueServer(tester=tester, worker_number=3, synchronous=True,
                                device=torch.device("cpu"))
    models = [{"weight": torch.full((1, 2), float(k)), "bias": torch.zeros(1)} for k in range(3)]
    server._set_prev_model(models[0])
    # no coalition members: every utility is the previous model's (no store needed)
    server.parameters = _Params()
    server._batch_size = lambda: 2
    assert tester.accuracy_metric.value is None
    got = server.evaluate_subsets([(), (), ()])
    assert tester.calls == ["async"] * 3
    # the tester's accuracy metric is left as get_metric leaves it
    assert tester.accuracy_metric.value == got[-1]
    want = []
    for _ in range(3):
        want.append(FedServer.get_metric(server, server.prev_model))
    assert got == want
    server.get_metric = lambda model, metric_type="acc": 0.5  # replaced on the instance
    assert server.evaluate_subsets([()]) == [0.5]
