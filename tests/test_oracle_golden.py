"""Pin the CPU oracle against the golden vectors recorded from the reference."""
import numpy as np
import pytest

from oracle import fedavg, quant, shapley, sign
from oracle import _c
from tests import golden as G


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


def same_bits(a, b):
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    nan = np.isnan(a)
    return np.array_equal(nan, np.isnan(b)) and np.array_equal(bits(a)[~nan], bits(b)[~nan])


@pytest.fixture(scope="module")
def fed():
    return G.load("fedavg.npz")


def test_fedavg_full_round_bit_exact(fed):
    for case in G.meta(fed):
        k = case["key"]
        U, n, order = fed[f"{k}_U"], fed[f"{k}_n"], fed[f"{k}_order"]
        assert same_bits(fedavg.fedavg_reference_order(U, n, order), fed[f"{k}_full"])
        assert same_bits(_c.fedavg_ref(U, n, order), fed[f"{k}_full"])


def test_fedavg_subsets_bit_exact(fed):
    for case in G.meta(fed):
        k = case["key"]
        U, n = fed[f"{k}_U"], fed[f"{k}_n"]
        for si in range(case["nsub"]):
            ids = fed[f"{k}_sub{si}_ids"]
            ref = fed[f"{k}_sub{si}_out"]
            assert same_bits(fedavg.fedavg_reference_order(U, n, ids), ref), (k, si)
            assert same_bits(_c.fedavg_ref(U, n, ids), ref), (k, si)


def test_fedavg_order_matters(fed):
    """Reversing the client order changes bits: the kernel must keep the order."""
    U, n, order = fed["c1_U"], fed["c1_n"], fed["c1_order"]
    rev = fedavg.fedavg_reference_order(U, n, order[::-1])
    assert not same_bits(rev, fed["c1_full"])
    ex = fedavg.fedavg_weighted(U, n, order)
    assert np.linalg.norm(rev - ex) / np.linalg.norm(ex) < 1e-6


def test_fedavg_torch_cpu_restatement(fed):
    import torch
    for case in G.meta(fed):
        k = case["key"]
        U, n, order = fed[f"{k}_U"], fed[f"{k}_n"], fed[f"{k}_order"]
        clients = [{nm: torch.from_numpy(v.copy()) for nm, v in G.split(U[i], case["layout"]).items()}
                   for i in range(U.shape[0])]
        out = fedavg.fedavg_torch_cpu(clients, n, order)
        flat = np.concatenate([out[nm].reshape(-1).numpy() for nm, _ in case["layout"]])
        assert same_bits(flat, fed[f"{k}_full"])


def test_sign_vote_bit_exact():
    z = G.load("sign_vote.npz")
    for case in G.meta(z):
        S, vote = z[f"{case['key']}_signs"], z[f"{case['key']}_vote"]
        assert same_bits(sign.majority_vote(S), vote)
        assert same_bits(sign.vote_from_counts(sign.vote_counts(S)), vote)


def test_sign_pack_layout_roundtrip():
    rng = np.random.default_rng(0)
    x = np.sign(rng.standard_normal(1000)).astype(np.float32)
    x[::17] = 0
    x[5] = np.nan
    planes = sign.pack_planes(x)
    assert planes.size == 4 * 8
    w = planes.reshape(-1, 2)
    for p in (0, 1, 2, 3, 4, 63, 64, 255, 256, 511, 999):
        g, j = divmod(p, 64)
        pos = (int(w[g, 0]) >> j) & 1
        neg = (int(w[g, 1]) >> j) & 1
        if np.isnan(x[p]):
            assert pos == 1 and neg == 1
        else:
            assert pos == int(x[p] > 0) and neg == int(x[p] < 0)
    assert same_bits(sign.unpack_planes(planes, 1000), x)
    assert np.all(w[1000 // 64 + 1:] == 0) and (int(w[15, 0]) >> 40) == 0


def test_sign_worker_bit_exact():
    z = G.load("sign_worker.npz")
    for case in G.meta(z):
        k, cfg = case["key"], case["cfg"]
        layout = case["layout"]
        p = z[f"{k}_p0"].copy()
        bufs = {}
        seen = set()
        for s in range(case["steps"]):
            grad, has = z[f"{k}_s{s}_grad"], z[f"{k}_s{s}_hasgrad"]
            vote = z[f"{k}_s{s}_vote"]
            off = 0
            new_p = p.copy()
            for ti, (name, shape) in enumerate(layout):
                m = int(np.prod(shape))
                sl = slice(off, off + m)
                off += m
                if not has[ti]:
                    continue
                first = name not in seen
                d, b = sign.worker_direction(grad[sl], bufs.get(name), first, cfg["momentum"],
                                             cfg["dampening"], cfg["nesterov"])
                if cfg["momentum"] != 0:
                    bufs[name] = b
                    seen.add(name)
                assert same_bits(sign.worker_sign(d), z[f"{k}_s{s}_sent"][sl]), (k, s, name)
                new_p[sl] = sign.worker_apply(p[sl], vote[sl], cfg["lr"], cfg["weight_decay"])
                if cfg["momentum"] != 0:
                    assert same_bits(bufs[name], z[f"{k}_s{s}_buf"][sl]), (k, s, name)
            p = new_p
            assert same_bits(p, z[f"{k}_s{s}_param"]), (k, s)


def test_dequant_bit_exact():
    z = G.load("dequant.npz")
    case = G.meta(z)[0]
    layout, K = case["layout"], case["K"]
    clients = []
    for i in range(K):
        c, parts = {}, []
        for name, shape in layout:
            if name in case["qnames"]:
                t = (z[f"q{i}_{name}_int"], z[f"q{i}_{name}_scale"], z[f"q{i}_{name}_zp"])
                c[name] = t
                parts.append(quant.dequant_channel(*t).reshape(-1))
            else:
                c[name] = z[f"q{i}_{name}_f32"]
                parts.append(c[name].reshape(-1))
        assert same_bits(np.concatenate(parts), z[f"deq{i}"]), i
        clients.append(c)
    agg = quant.dequant_fedavg(clients, z["n"], list(range(K)), layout)
    assert same_bits(agg, z["agg"])


def test_quantize_matches_torch_formula():
    z = G.load("quantize.npz")
    q = quant.quantize_affine(z["pt_x"], float(z["pt_scale"]), int(z["pt_zp"]))
    assert np.array_equal(q, z["pt_q"].astype(np.int64))
    qt = quant.quantize_affine(z["tie_x"], 0.0625, 10)
    assert np.array_equal(qt, z["tie_q"].astype(np.int64))
    qc = quant.quantize_per_channel(z["pc_x"], z["pc_scale"], np.zeros(12, np.int64))
    assert np.array_equal(qc, z["pc_q"].astype(np.int64))


def _shapley_setup(case):
    layout = [(nm, tuple(s)) for nm, s in case["layout"]]
    U = np.array(case["U"], np.float32)
    n = case["n"]
    prev = np.array(case["prev"], np.float32)
    target = np.array(case["target"], np.float64)

    def subset_model(subset):
        if not subset:
            return prev
        return fedavg.fedavg_reference_order(U, n, subset)

    def metric(model):
        d = np.asarray(model, np.float64) - target
        return float(1.0 / (1.0 + float(np.dot(d, d)) / case["scale"]))

    return layout, U, n, prev, subset_model, metric


def test_multiround_shapley_golden():
    for case in G.shapley_cases():
        if not case["tag"].startswith("multiround"):
            continue
        _, U, n, _, subset_model, metric = _shapley_setup(case)
        sv, metrics = shapley.multiround_shapley(case["K"], subset_model, metric)
        for k, v in case["sv"].items():
            assert abs(sv[int(k)] - v) <= 1e-12
        assert [list(s) for s in metrics.keys()] == case["evaluated"]


def test_gtg_shapley_golden():
    for case in G.shapley_cases():
        if not case["tag"].startswith("gtg"):
            continue
        _, U, n, prev, subset_model, metric = _shapley_setup(case)
        agg = fedavg.fedavg_reference_order(U, n, range(case["K"]))
        np.random.seed(case["seed"])
        sv, evaluated = shapley.gtg_shapley(case["K"], prev, agg, subset_model, metric)
        for k, v in case["sv"].items():
            assert abs(sv[int(k)] - v) <= 1e-12
        assert [list(s) for s in evaluated] == case["evaluated"]


@pytest.mark.parametrize("b", [1.0, 3.0, 7.0, 550.0, 55000.0, 16777215.0, 33554432.0, 123457.0,
                               2147483648.0])
def test_kernel_fast_division_exhaustive(b):
    """The kernels' guarded fp32 division equals IEEE a/b for every mantissa."""
    assert _c.fastdiv_check(b) == 0
