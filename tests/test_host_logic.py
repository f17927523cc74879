"""CPU tests of the host logic (round protocol, stores, layouts, queue, Shapley
scheduling) with the kernels replaced by numpy test doubles (tests/cpu_doubles.py)."""
import threading

import numpy as np
import pytest
import torch

from oracle import _c
from tests import cpu_doubles
from tests import golden as G

CPU = torch.device("cpu")


def same_bits(a, b):
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    nan = np.isnan(a)
    return np.array_equal(nan, np.isnan(b)) and np.array_equal(
        a.view(np.uint32)[~nan], b.view(np.uint32)[~nan])


@pytest.fixture
def doubles(monkeypatch):
    cpu_doubles.install(monkeypatch)


def test_layout_alignment_and_views():
    from distributed_learning_simulator_amd.layout import ParameterLayout
    from distributed_learning_simulator_amd.model_shapes import resnet18_cifar
    lay = ParameterLayout(resnet18_cifar())
    assert lay.numel == 11173962 and len(lay) == 62
    assert all(o % 64 == 0 for o in lay.offsets) and lay.P % 64 == 0
    d = {n: torch.randn(s) for n, s in resnet18_cifar()}
    row = lay.flatten(d)
    v = lay.views(row)
    assert all(torch.equal(v[n], d[n]) for n in d)
    assert lay.matches(d) and not lay.matches(dict(list(d.items())[1:]))


def test_quant_layout_tiles():
    from distributed_learning_simulator_amd.quant_store import QuantLayout
    payload = {"w": (torch.zeros(5, 9, dtype=torch.int8), torch.ones(5), torch.zeros(5)),
               "b": torch.zeros(5),
               "u": (torch.zeros(3, 5000, dtype=torch.uint8), torch.ones(3), torch.zeros(3)),
               "v": (torch.zeros(6, 3, dtype=torch.int8), torch.ones(6), torch.zeros(6))}
    ql = QuantLayout(payload)
    t, nfast = ql.tiles()
    assert t["len"].max() <= 1024 and all(d % 16 == 0 for d in t["dst"])
    # the 15 1 KiB tiles of the 3x5000 "u" lie in one channel except those starting
    # at 4096 and 9216 (cut into small tiles); "w" (rows of 9): one small tile;
    # "b": one fp32 tile; "v" (rows of 3): a general tile
    g = np.cumsum((0,) + nfast)
    one = t[:g[4]]
    assert all(r["kind"] != 0 and r["row_pos"] + r["len"] <= r["row_len"] for r in one)
    assert t[g[8]:g[9]]["kind"].tolist() == [0]
    small, rest = t[g[9]:g[10]], t[g[10]:]
    assert all(int(r["len"]) <= 256 and int(r["row_len"]) >= 4 for r in small)
    assert rest["kind"].tolist() == [1] and int(rest[0]["row_len"]) == 3
    assert nfast == (0, 0, 0, 13, 0, 0, 0, 0, 1, 1 + 4 + 4)
    assert sum(int(r["len"]) for r in t) == 45 + 5 + 15000 + 18
    u = t[t["kind"] == 2]
    assert all(int(r["row_pos"]) == int(r["src"] - ql.src[2]) % 5000 for r in u)
    assert all(int(r["chan0"]) == 5 + int(r["src"] - ql.src[2]) // 5000 for r in u)
    assert ql.matches(payload)


@pytest.mark.parametrize("lane_tile", [1024, "adaptive"])
def test_quant_layout_channel_aligned_tiles(lane_tile, monkeypatch):
    """Long channel rows (multiple of 64, last 1 KiB slice at least 7/8 full) get
    channel-aligned tiles of up to 4096 elements, grouped by slice count; other
    int tensors with rows a multiple of 16 get multi-channel (lane) tiles from their
    start: LANE_TILE elements, or adaptive (the width with the fewest tiles of at
    most 4 channel rows: 4 KiB for conv and mid, 4 rows = 256 elements for pw)."""
    from distributed_learning_simulator_amd import quant_store
    from distributed_learning_simulator_amd.quant_store import QuantLayout
    monkeypatch.setattr(quant_store, "LANE_TILE", lane_tile)
    LANE_TILE = 4096 if lane_tile == "adaptive" else lane_tile
    shapes = {"fc": (3, 25088), "conv": (2, 512, 3, 3), "mid": (4, 256, 3, 3), "k": (2, 1024),
              "c1": (5, 3, 3, 3), "pw": (8, 64, 1, 1)}
    payload = {k: (torch.zeros(s, dtype=torch.int8), torch.ones(s[0]), torch.zeros(s[0]))
               for k, s in shapes.items()}
    ql = QuantLayout(payload)
    t, nfast = ql.tiles()
    # fc: 6 x 4096 + 512 per channel (2 % idle lanes); k: 1024; conv (row 4608:
    # 11 % idle lanes in its last slice) and mid (row 2304): lane tiles of
    # LANE_TILE from their start; c1 (row 27): general 1 KiB tiles
    if lane_tile == 1024:  # pw: one 512-element lane tile over 8 channel rows
        assert nfast[:8] == (3 * 6, 0, 0, 3 + 2, 0, 0, 0, 9 + 9 + 1) and nfast[8] == 0
        assert nfast[9] == (5 * 27 + 255) // 256  # c1 (rows of 27): small tiles
    else:  # 9216-element tensors: 4096 + 4096 + 1024; pw: 2 x 4 rows of 64
        assert nfast[:8] == (3 * 6, 0, 0, 3 + 2, 2 + 2, 0, 0, 1 + 1 + 2) and nfast[8] == 0
        lanes = t[sum(nfast[:4]):sum(nfast[:8])]
        # at most 4 channel rows per lane tile (the FMA kernel's staged table)
        assert max((int(r["row_pos"]) + int(r["len"]) - 1) // int(r["row_len"]) + 1
                   for r in lanes) <= 4
        assert nfast[9] == (5 * 27 + 255) // 256  # c1 (rows of 27): small tiles
    nf = sum(nfast)
    one = t[:sum(nfast[:4])]
    sl = [(int(r["len"]) + 1023) // 1024 for r in one]
    assert sl == sorted(sl, reverse=True)
    assert all(r["row_pos"] + r["len"] <= r["row_len"] for r in one)
    lanes = t[sum(nfast[:4]):sum(nfast[:8])]
    assert all(int(r["row_len"]) % 16 == 0 and int(r["len"]) <= LANE_TILE for r in lanes)
    assert all(d % 16 == 0 for d in t["dst"]) and all(s % 16 == 0 for s in t["src"])
    assert nf == len(t)  # no general tiles
    for i, name in enumerate(ql.names):  # every element of every tensor exactly once
        mine = t[(t["dst"] >= ql.layout.offsets[i]) &
                 (t["dst"] < ql.layout.offsets[i] + ql.layout.numels[i])]
        cover = np.zeros(ql.layout.numels[i], np.int32)
        for r in mine:
            e = int(r["dst"]) - ql.layout.offsets[i]
            cover[e:e + int(r["len"])] += 1
            assert int(r["src"]) - ql.src[i] == e
            assert int(r["chan0"]) == ql.chan_base[i] + e // ql.row_len[i]
            assert int(r["row_pos"]) == e % ql.row_len[i]
        assert (cover == 1).all(), name


def test_repeated_result_served_once_per_consumer():
    from distributed_learning_simulator_amd.task_queue import RepeatedResult, ThreadTaskQueue
    q = ThreadTaskQueue(worker_fun=lambda task, _: RepeatedResult(task, num=3) if task else None)
    q.put_result(RepeatedResult("r0", num=3))
    got = {}

    def consumer(i):
        a = q.get_result(timeout=10)
        if i == 0:  # the fast worker asks again before the others took r0
            q.add_task("r1")
        b = q.get_result(timeout=10)
        got[i] = (a, b)

    ts = [threading.Thread(target=consumer, args=(i,)) for i in range(3)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(20)
    q.stop()
    assert got == {i: ("r0", "r1") for i in range(3)}


def test_queue_surfaces_server_errors():
    from distributed_learning_simulator_amd.task_queue import ThreadTaskQueue

    def boom(task, _):
        raise ValueError("bad payload")
    q = ThreadTaskQueue(worker_fun=boom)
    q.add_task(1)
    with pytest.raises(RuntimeError):
        q.get_result(timeout=10)
    q.stop()


def test_factory_names_and_errors():
    from distributed_learning_simulator_amd import factory
    with pytest.raises(RuntimeError, match="unknown algorithm"):
        factory.get_server("fedprox", tester=None, worker_number=1)
    with pytest.raises(RuntimeError, match="unknown algorithm"):
        factory.get_worker("fedprox")


def test_fed_server_round_protocol(doubles):
    from distributed_learning_simulator_amd.servers.fed_server import FedServer
    z = G.load("fedavg.npz")
    case = G.meta(z)[0]
    k, layout = case["key"], case["layout"]
    U, n, order = z[f"{k}_U"], z[f"{k}_n"], z[f"{k}_order"]
    server = FedServer(tester=None, worker_number=case["K"], synchronous=True, device=CPU)
    for wid in order:
        d = {nm: torch.from_numpy(v.copy()) for nm, v in G.split(U[wid], layout).items()}
        server.worker_data_queue.add_task((int(wid), int(n[wid]), d))
    for w in range(case["K"]):
        server.worker_data_queue.get_result(consumer=w)
    res = server.worker_data_queue.get_result(consumer=0)
    flat = np.concatenate([res[nm].reshape(-1).numpy() for nm, _ in layout])
    assert same_bits(flat, z[f"{k}_full"])
    assert server.round == 1 and len(server.parameters) == 0
    # subsets / empty subset through the public hook
    for wid in order:
        d = {nm: torch.from_numpy(v.copy()) for nm, v in G.split(U[wid], layout).items()}
        server.parameters[int(wid)] = (int(n[wid]), d)
    ids = z[f"{k}_sub4_ids"]
    sub = server.get_subset_model(tuple(int(i) for i in ids))
    flat = np.concatenate([sub[nm].reshape(-1).numpy() for nm, _ in layout])
    assert same_bits(flat, z[f"{k}_sub4_out"])
    assert server.get_subset_model(()) is server.prev_model


@pytest.mark.parametrize("method", ["exact", "gemm"])
def test_shapley_servers_host_logic(doubles, method, tmp_path):
    from distributed_learning_simulator_amd.servers.GTG_shapley_value_server import \
        GTGShapleyValueServer
    from distributed_learning_simulator_amd.servers.multiround_shapley_value_server import \
        MultiRoundShapleyValueServer
    for case in G.shapley_cases():
        layout = [(nm, tuple(s)) for nm, s in case["layout"]]
        K = case["K"]
        U = np.array(case["U"], np.float32)
        target = np.array(case["target"], np.float64)
        cls = GTGShapleyValueServer if case["tag"].startswith("gtg") else \
            MultiRoundShapleyValueServer
        kw = {} if cls is GTGShapleyValueServer else {"metric_dir": str(tmp_path)}
        server = cls(tester=None, worker_number=K, synchronous=True, device=CPU,
                     subset_method=method, **kw)
        server._set_prev_model(G.split(torch.tensor(case["prev"]), layout))

        def util(model, metric_type="acc", layout=layout, target=target, case=case):
            v = np.concatenate([np.asarray(model[nm], np.float64).reshape(-1) for nm, _ in layout])
            d = v - target
            return float(1.0 / (1.0 + float(np.dot(d, d)) / case["scale"]))

        server.get_metric = util
        np.random.seed(case["seed"])
        for i in range(K):
            d = {nm: torch.from_numpy(v.copy()) for nm, v in G.split(U[i], layout).items()}
            server.worker_data_queue.add_task((i, int(case["n"][i]), d))
        sv = server.shapley_values[1]
        tol = 1e-12 if method == "exact" else 1e-5
        for kk, v in case["sv"].items():
            assert abs(float(sv[int(kk)]) - v) <= tol, (case["tag"], kk)
        if method == "exact":
            assert {tuple(s) for s in server.evaluated_subsets} == \
                {tuple(s) for s in case["evaluated"]}


def test_sign_server_vote_and_nonternary(doubles):
    from distributed_learning_simulator_amd.servers.sign_sgd_server import SignSGDServer
    z = G.load("sign_vote.npz")
    case = G.meta(z)[0]
    S, vote = z["c0_signs"], z["c0_vote"]
    layout = case["layout"]
    server = SignSGDServer(tester=None, worker_number=case["K"], synchronous=True, device=CPU)
    for k in range(case["K"]):
        server.worker_data_queue.add_task(
            [torch.from_numpy(v.copy()) for v in G.split(S[k], layout).values()])
    res = server.worker_data_queue.get_result(consumer=0)
    assert same_bits(np.concatenate([t.reshape(-1).numpy() for t in res]), vote)
    # the reference's name-mangled hook is kept as an alias (D1)
    assert SignSGDServer._SignSGDServer__worker is SignSGDServer._process_worker_data
    bad = SignSGDServer(tester=None, worker_number=1, synchronous=True, device=CPU)
    with pytest.raises(ValueError, match="outside"):
        bad.worker_data_queue.add_task([torch.tensor([0.5, 1.0, -1.0])])


def test_fastdiv_random_divisors():
    rng = np.random.default_rng(1)
    for b in rng.integers(1, 2**31, size=3):
        assert _c.fastdiv_check(float(np.float32(b))) == 0


def test_union_order_topological_merge():
    """dls_subset_fedavg_union_f32 walks one client order for a whole batch; every
    coalition's own order must be a subsequence of it (aggregation.union_order)."""
    from distributed_learning_simulator_amd.aggregation import union_order
    assert union_order([[0, 2], [1, 2, 5], [0, 1]]) == [0, 1, 2, 5]
    assert union_order([[3, 1], [1, 0]]) == [3, 1, 0]  # rows need not be sorted
    assert union_order([[0, 1], [1, 0]]) is None  # contradictory orders
    assert union_order([[0, 0]]) is None  # a repeated client: per-coalition kernel
    rng = np.random.default_rng(0)
    for _ in range(50):
        perm = rng.permutation(40)  # arbitrary worker -> row map, sorted worker tuples
        subs = [[int(perm[w]) for w in sorted(rng.choice(40, rng.integers(1, 40), replace=False))]
                for _ in range(64)]
        order = union_order(subs)
        pos = {r: i for i, r in enumerate(order)}
        assert all(all(pos[a] < pos[b] for a, b in zip(s, s[1:])) for s in subs)


def test_union_batch_tables():
    from distributed_learning_simulator_amd.aggregation import union_batch
    subs = [[4, 2], [2, 7], [4, 7, 9]] + [[9]] * 61  # 64 coalitions: bit 63 set
    rows, w, member, tot = union_batch(subs, {2: 10, 4: 20, 7: 30, 9: 40}, CPU)
    assert rows.tolist() == [4, 2, 7, 9] and w.tolist() == [20, 10, 30, 40]
    m = [int(x) & (2**64 - 1) for x in member.tolist()]
    assert m[0] == 0b101 and m[1] == 0b011 and m[2] == 0b110
    assert m[3] == (1 << 2) | sum(1 << s for s in range(3, 64))
    assert list(tot)[:3] == [30.0, 40.0, 90.0]


def test_subset_models_union_path_matches_reference_order(doubles):
    """Store-level: the union path gives each coalition in its own order."""
    from distributed_learning_simulator_amd.aggregation import ClientUpdateStore
    from distributed_learning_simulator_amd.layout import ParameterLayout
    lay = ParameterLayout([("w", (5, 7)), ("b", (3,))])
    st = ClientUpdateStore(lay, CPU, capacity=6)
    g = torch.Generator().manual_seed(0)
    rows = [st.acquire() for _ in range(6)]
    for r in rows:
        st.write(r, {"w": torch.randn(5, 7, generator=g), "b": torch.randn(3, generator=g)})
    n = {r: 100 + 37 * r for r in rows}
    subs = [[rows[5], rows[0]], [rows[0], rows[3], rows[1]], [rows[2]]]
    out = st.subset_models(subs, n)
    U = st.U.numpy()
    for s, sub in enumerate(subs):
        assert same_bits(out[s].numpy(), _c.fedavg_ref(U, [n.get(i, 1) for i in range(6)], sub))


@pytest.mark.parametrize("tag", ["gtg_50_4", "multiround_12"])
def test_shapley_host_logic_config5_scale(doubles, tag, tmp_path):
    """Host logic at config 5's client count (GTG N=50, multiround N=12) with the
    kernel doubles: SV within 1e-12, same coalitions, metric_1 pickle bytes."""
    from distributed_learning_simulator_amd.servers.GTG_shapley_value_server import \
        GTGShapleyValueServer
    from distributed_learning_simulator_amd.servers.multiround_shapley_value_server import \
        MultiRoundShapleyValueServer
    case = next(c for c in G.shapley_large_cases() if c["tag"] == tag)
    layout = [(nm, tuple(s)) for nm, s in case["layout"]]
    K = case["K"]
    target = case["target"]
    gtg = tag.startswith("gtg")
    cls = GTGShapleyValueServer if gtg else MultiRoundShapleyValueServer
    kw = {} if gtg else {"metric_dir": str(tmp_path)}
    server = cls(tester=None, worker_number=K, synchronous=True, device=CPU, **kw)
    server._set_prev_model(G.split(torch.tensor(case["prev"]), layout))

    def util(model, metric_type="acc"):
        v = np.concatenate([np.asarray(model[nm], np.float64).reshape(-1) for nm, _ in layout])
        d = v - target
        return float(1.0 / (1.0 + float(np.dot(d, d)) / case["scale"]))

    server.get_metric = util
    np.random.seed(case["seed"])
    for i in range(K):
        d = {nm: torch.from_numpy(v.copy()) for nm, v in G.split(case["U"][i], layout).items()}
        server.worker_data_queue.add_task((i, int(case["n"][i]), d))
    sv = server.shapley_values[1]
    for kk, v in case["sv"].items():
        assert abs(float(sv[int(kk)]) - v) <= 1e-12, kk
    assert {tuple(s) for s in server.evaluated_subsets} == set(case["evaluated"])
    if not gtg:
        assert (tmp_path / "metric_1").read_bytes() == case["metric_pickle"]


@pytest.mark.parametrize("tag", ["gtg_50_4", "multiround_12"])
def test_shapley_host_logic_config5_gemm_method(doubles, tag, tmp_path):
    """subset_method="gemm" host logic at config 5's client count with the GEMM
    double (fp64 product rounded to fp32, not the reference's op order): SV
    within 1e-5 and the identical client ranking (north_star tolerance)."""
    from distributed_learning_simulator_amd.servers.GTG_shapley_value_server import \
        GTGShapleyValueServer
    from distributed_learning_simulator_amd.servers.multiround_shapley_value_server import \
        MultiRoundShapleyValueServer
    case = next(c for c in G.shapley_large_cases() if c["tag"] == tag)
    layout = [(nm, tuple(s)) for nm, s in case["layout"]]
    K = case["K"]
    target = case["target"]
    gtg = tag.startswith("gtg")
    cls = GTGShapleyValueServer if gtg else MultiRoundShapleyValueServer
    kw = {} if gtg else {"metric_dir": str(tmp_path)}
    server = cls(tester=None, worker_number=K, synchronous=True, device=CPU,
                 subset_method="gemm", **kw)
    server._set_prev_model(G.split(torch.tensor(case["prev"]), layout))

    def util(model, metric_type="acc"):
        v = np.concatenate([np.asarray(model[nm], np.float64).reshape(-1) for nm, _ in layout])
        d = v - target
        return float(1.0 / (1.0 + float(np.dot(d, d)) / case["scale"]))

    server.get_metric = util
    np.random.seed(case["seed"])
    for i in range(K):
        d = {nm: torch.from_numpy(v.copy()) for nm, v in G.split(case["U"][i], layout).items()}
        server.worker_data_queue.add_task((i, int(case["n"][i]), d))
    sv = server.shapley_values[1]
    ref = {int(k): v for k, v in case["sv"].items()}
    for k, v in ref.items():
        assert abs(float(sv[k]) - v) <= 1e-5, k
    assert sorted(ref, key=ref.get) == sorted(sv, key=lambda k: float(sv[k]))


def test_data_serialization_size_matches_pickle():
    """The compression-ratio sizes (ref servers/fed_quant_server.py:41-42,
    workers/fed_quant_worker.py:28-30,43) are len(pickle.dumps(payload)) of the
    CPU payload, whatever its values."""
    import pickle

    from distributed_learning_simulator_amd.model_util import get_data_serialization_size
    g = torch.Generator().manual_seed(3)
    params = {"conv.weight": torch.randn(16, 3, 3, 3, generator=g), "fc.bias": torch.randn(10, generator=g)}
    q = {"conv.weight": (torch.randint(-128, 128, (16, 3, 3, 3), dtype=torch.int8, generator=g),
                         torch.rand(16, generator=g), torch.zeros(16, dtype=torch.int32)),
         "fc.bias": torch.randn(10, generator=g)}
    for data in (params, q, (torch.zeros(100, dtype=torch.uint8), torch.ones(3), torch.zeros(3, dtype=torch.int32))):
        assert get_data_serialization_size(data) == len(pickle.dumps(data))
    assert get_data_serialization_size(q) < get_data_serialization_size(params)


def test_sliced_store_write_views_row():
    """SlicedClientUpdateStore (the bit-exact sharded exchange's slice-major rows):
    a dict written tensor by tensor across slice boundaries reads back exactly,
    as views / copies and as a flat row; block B[d] is slice d of every row."""
    from distributed_learning_simulator_amd.aggregation import SlicedClientUpdateStore
    from distributed_learning_simulator_amd.distributed import slice_bounds
    from distributed_learning_simulator_amd.layout import ParameterLayout
    shapes = [("a", (3, 50)), ("b", (7,)), ("c", (4, 4, 9)), ("d", (130,))]
    layout = ParameterLayout(shapes)
    for world in (1, 2, 3, 5):
        L = slice_bounds(layout.P, world)[1]
        st = SlicedClientUpdateStore(layout, "cpu", 1, world, L)
        g = torch.Generator().manual_seed(world)
        ds = [{n: torch.randn(s, generator=g) for n, s in shapes} for _ in range(3)]
        rows = [st.acquire() for _ in ds]  # grows past capacity 1
        for r, d in zip(rows, ds):
            st.write(r, d)
        for r, d in zip(rows, ds):
            v = st.views(r)
            flat = layout.flatten(d)
            assert torch.equal(st.row(r), flat)
            for n, _ in shapes:
                assert torch.equal(v[n], d[n])
            for s_ in range(world):
                assert torch.equal(st.B[s_, r], torch.cat([flat, torch.zeros(world * L - layout.P)])
                                   [s_ * L:(s_ + 1) * L])


def test_quant_column_chunks_cutting_lane_tiles(doubles):
    """ADVICE r05 (host side; tests/test_gpu_quant.py runs the kernels): column
    sub-tables keep the tiles that start in their range, so a chunk bound inside a
    multi-channel lane tile leaves that tile to the chunk before it, which writes
    past the bound; run in order, the chunks give the whole table's bits."""
    from distributed_learning_simulator_amd.quant_store import QTILE_DTYPE, QuantizedClientStore
    g = torch.Generator().manual_seed(77)
    shapes = {"l1": (8, 64, 3, 3), "fc": (3, 4096), "pw": (32, 64, 1, 1)}
    payloads, n = [], [37, 211, 5]
    for _ in range(3):
        p = {}
        for name, s_ in shapes.items():
            p[name] = (torch.randint(-128, 128, s_, generator=g, dtype=torch.int8),
                       torch.rand(s_[0], generator=g, dtype=torch.float64) * 1e-2 + 1e-4,
                       torch.zeros(s_[0], dtype=torch.int64))
        payloads.append(p)
    store = QuantizedClientStore(payloads[0], CPU, capacity=3)
    rows = []
    for p in payloads:
        r = store.acquire()
        store.write(r, p)
        rows.append(r)
    P = store.layout.P
    whole = store.fedavg(rows, n, out=torch.full((P,), float("nan")))
    t = store.tiles.numpy().view(QTILE_DTYPE)[:store.ntiles]
    lanes = t[sum(store.nfast[:4]):sum(store.nfast[:8])]
    wide = lanes[lanes["len"] >= 64]
    cuts = sorted({int(wide[0]["dst"]) + 16, int(wide[-1]["dst"]) + 48})
    out = torch.full((P,), float("nan"))
    crossing = 0
    for c0, c1 in zip([0] + cuts, cuts + [P]):
        sub, nsub, _ = store.table(cols=(c0, c1))
        st = sub.numpy().view(QTILE_DTYPE)[:nsub]
        crossing += int(((st["dst"] + st["len"]) > c1).sum())
        store.fedavg(rows, n, out=out, cols=(c0, c1))
    assert crossing >= len(cuts)
    assert same_bits(out.numpy(), whole.numpy())


def test_aggregation_mode_from_the_command_line(doubles):
    """a reference user selects the FMA aggregation (the
    fed_quant path that meets the 80 % HBM bar) with a flag, no code change:
    simulator --aggregation_mode fma reaches the server the factory builds."""
    from distributed_learning_simulator_amd import factory
    from distributed_learning_simulator_amd.simulator import get_config, server_kwargs
    base = ["--worker_number", "2", "--round", "1"]
    cfg = get_config(["--distributed_algorithm", "fed_quant", "--aggregation_mode", "fma"] + base)
    assert cfg.aggregation_mode == "fma" and server_kwargs(cfg) == {"aggregation_mode": "fma"}
    assert cfg.tester_conv == "dls"
    assert get_config(["--distributed_algorithm", "fed", "--tester_conv", "miopen"] + base).tester_conv == "miopen"
    server = factory.get_server("fed_quant", tester=None, worker_number=2, synchronous=True,
                                device=CPU, **server_kwargs(cfg))
    assert server.aggregation_mode == "fma"
    server.stop()
    assert get_config(["--distributed_algorithm", "fed"] + base).aggregation_mode == "exact"
    assert server_kwargs(get_config(["--distributed_algorithm", "sign_SGD"] + base)) == {}
    with pytest.raises(SystemExit):
        get_config(["--distributed_algorithm", "fed", "--aggregation_mode", "tree"] + base)
    with pytest.raises(ValueError, match="aggregation_mode"):
        factory.get_server("fed", tester=None, worker_number=2, synchronous=True, device=CPU,
                           aggregation_mode="tree")


def test_split_forward_batch_rule():
    """the utility forward's batch is capped by a memory budget; the
    tester's batch_size only raises it when it fits (the rule
    Inferencer.split_batch applies; GPU test: test_gpu_conv.py)."""
    from distributed_learning_simulator_amd.models import ResNet18
    from distributed_learning_simulator_amd.trainer import split_forward_batch
    per = ResNet18().split_activation_bytes(32, 32)
    assert per == 4 * 3 * 32 * 32 + 16 * 64 * 32 * 32  # input + 4 layer1 activations
    assert ResNet18().split_activation_bytes(224, 224) > 40 * per
    assert split_forward_batch(10000, 1000, 10000, per, 70e9) == 10000
    assert split_forward_batch(500, 1000, 10000, per, 70e9) == 500
    assert split_forward_batch(10000, 1000, 10000, per, 2e9) == int(2e9 // per)
    assert split_forward_batch(10000, 20000, 10000, per, 70e9) == 10000
    assert split_forward_batch(10000, 1000, 10000, per, 10) == 1
