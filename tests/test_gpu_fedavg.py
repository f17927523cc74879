"""GPU parity: FedAvg / subset kernels (through the C-ABI) vs the oracle and golden vectors."""
import numpy as np
import pytest
import torch

from oracle import _c, fedavg as ofed
from tests import golden as G

pytestmark = pytest.mark.gpu

dev = torch.device("cuda")


def same_bits(a, b):
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    nan = np.isnan(a)
    return np.array_equal(nan, np.isnan(b)) and np.array_equal(
        a.view(np.uint32)[~nan], b.view(np.uint32)[~nan])


def pad4(U):
    K, P = U.shape
    Pp = (P + 3) // 4 * 4
    out = np.zeros((K, Pp), np.float32)
    out[:, :P] = U
    return out


def run_fedavg(U, rows, n, mode=0):
    from distributed_learning_simulator_amd import _native
    Ud = torch.from_numpy(pad4(U)).to(dev)
    P = Ud.shape[1]
    out = torch.empty(P, dtype=torch.float32, device=dev)
    rows_t = torch.tensor(list(rows), dtype=torch.int32, device=dev)
    w = torch.tensor([int(n[r]) for r in rows], dtype=torch.float32, device=dev)
    _native.fedavg(Ud, rows_t, w, float(sum(int(n[r]) for r in rows)), P, out, mode=mode)
    return out.cpu().numpy()[: U.shape[1]]


def test_fedavg_golden_bit_exact():
    z = G.load("fedavg.npz")
    for case in G.meta(z):
        k = case["key"]
        U, n, order = z[f"{k}_U"], z[f"{k}_n"], z[f"{k}_order"]
        assert same_bits(run_fedavg(U, order, n), z[f"{k}_full"]), k
        for si in range(case["nsub"]):
            ids = z[f"{k}_sub{si}_ids"]
            assert same_bits(run_fedavg(U, ids, n), z[f"{k}_sub{si}_out"]), (k, si)


@pytest.mark.parametrize("K,P", [(1, 8), (3, 1028), (9, 4096 * 3 + 12), (64, 1036), (65, 2052),
                                 (100, 1 << 18), (131, 4100), (257, 1028),
                                 (3, (1 << 22) + 1036), (65, (1 << 22) + 64 * 1024 + 12),
                                 (7, 2_400_004), (5, 2_000_000)])
def test_fedavg_random_bit_exact(K, P):
    g = torch.Generator().manual_seed(K * 7 + P)
    U = (torch.randn(K, P, generator=g) * 0.05).numpy()
    U[0, :8] = [0.0, -0.0, 1e-40, -1e-39, 3e38, np.inf, np.nan, 1e-45]
    n = [int(x) for x in torch.randint(1, 1001, (K,), generator=g)]
    order = [int(x) for x in torch.randperm(K, generator=g)]
    assert same_bits(run_fedavg(U, order, n), _c.fedavg_ref(U, n, order))


def test_fedavg_resnet18_k100_bit_exact():
    """BASELINE config 2 at full size: 100 x 11,173,962 fp32, bit-exact."""
    K, P = 100, 11173962
    g = torch.Generator(device=dev).manual_seed(20250128)
    Ud = torch.randn(K, (P + 3) // 4 * 4, generator=g, device=dev) * 0.05
    n = [100 + (7 * i) % 901 for i in range(K)]
    order = list(range(K))[::-1]
    from distributed_learning_simulator_amd import _native
    out = torch.empty(Ud.shape[1], dtype=torch.float32, device=dev)
    _native.fedavg(Ud, torch.tensor(order, dtype=torch.int32, device=dev),
                   torch.tensor([n[r] for r in order], dtype=torch.float32, device=dev),
                   float(sum(n)), Ud.shape[1], out)
    U = Ud.cpu().numpy()
    ref = _c.fedavg_ref(U, n, order)
    assert same_bits(out.cpu().numpy(), ref)


def test_fedavg_fma_mode_normwise():
    K, P = 64, 1 << 16
    g = torch.Generator().manual_seed(3)
    U = (torch.randn(K, P, generator=g) * 0.05).numpy()
    n = [int(x) for x in torch.randint(100, 1001, (K,), generator=g)]
    got = run_fedavg(U, range(K), n, mode=1)
    ex = ofed.fedavg_weighted(U, n, range(K))
    assert np.linalg.norm(got - ex) / np.linalg.norm(ex) < 1e-6  # north-star tolerance


def test_subset_exact_batched_matches_oracle():
    from distributed_learning_simulator_amd import _native
    K, P = 12, 8192 + 4
    g = torch.Generator().manual_seed(5)
    U = (torch.randn(K, P, generator=g) * 0.05).numpy()
    n = [int(x) for x in torch.randint(100, 1001, (K,), generator=g)]
    subsets = [[0], [1, 3], [2, 5, 7, 11], list(range(K)), [11, 0, 4]]
    off, rows, w, tot = [0], [], [], []
    for s in subsets:
        rows += s
        w += [n[r] for r in s]
        tot.append(float(sum(n[r] for r in s)))
        off.append(len(rows))
    Ud = torch.from_numpy(U).to(dev)
    out = torch.empty((len(subsets), P), dtype=torch.float32, device=dev)
    _native.subset_fedavg(Ud, torch.tensor(off, dtype=torch.int32, device=dev),
                          torch.tensor(rows, dtype=torch.int32, device=dev),
                          torch.tensor(w, dtype=torch.float32, device=dev),
                          torch.tensor(tot, dtype=torch.float32, device=dev), P, out)
    got = out.cpu().numpy()
    for i, s in enumerate(subsets):
        assert same_bits(got[i], _c.fedavg_ref(U, n, s)), i


@pytest.mark.parametrize("S,K,P", [(1, 1, 128), (5, 7, 1000), (50, 50, 131072 + 64), (64, 50, 4096),
                                   (70, 300, 2048), (45, 300, 2048 + 64), (52, 17, 4096 + 192),
                                   (33, 2, 640)])
def test_subset_gemm_mfma_normwise(S, K, P):
    """fp32 MFMA contraction vs fp64: normwise <= 1e-6 (north-star tolerance);
    45 x 300: the running sums of a second client chunk; 52 x 17: odd K; 33 x 2:
    a second M tile of one row."""
    from distributed_learning_simulator_amd import _native
    g = torch.Generator().manual_seed(S * 1000 + K)
    U = torch.randn(K + 3, P, generator=g) * 0.05
    rows = torch.randperm(K + 3, generator=g)[:K]
    C = torch.rand(S, K, generator=g, dtype=torch.float64)
    C = (C * (torch.rand(S, K, generator=g) < 0.6)).double()
    C[:, 0] += 0.1
    C = C / C.sum(1, keepdim=True)
    out = torch.full((S, P), float("nan"), device=dev)
    _native.subset_gemm(C.float().to(dev), U.to(dev), rows.int().to(dev), P, out)
    ref = C @ U[rows].double()
    got = out.cpu().double()
    err = torch.linalg.norm(got - ref, dim=1) / torch.linalg.norm(ref, dim=1)
    assert float(err.max()) < 1e-6, float(err.max())


def test_subset_gemm_asymmetric_layout_check():
    """A = I-like coefficients with an asymmetric U catch any row/col swap."""
    from distributed_learning_simulator_amd import _native
    K, P = 40, 256
    U = torch.arange(K * P, dtype=torch.float32).reshape(K, P) / 1000.0
    C = torch.eye(K)[:33]  # S=33 -> two M tiles, last one nearly empty
    out = torch.empty((33, P), device=dev)
    _native.subset_gemm(C.to(dev), U.to(dev), torch.arange(K, dtype=torch.int32, device=dev), P,
                        out)
    assert torch.equal(out.cpu(), U[:33])


def test_fed_server_round_golden():
    """End to end through the drop-in FedServer (arrival order, dict views)."""
    from distributed_learning_simulator_amd.servers.fed_server import FedServer
    z = G.load("fedavg.npz")
    case = G.meta(z)[1]
    k, layout = case["key"], case["layout"]
    U, n, order = z[f"{k}_U"], z[f"{k}_n"], z[f"{k}_order"]

    server = FedServer(tester=None, worker_number=case["K"], multi_process=False, synchronous=True)
    res = None
    for wid in order:
        d = {nm: torch.from_numpy(v.copy()) for nm, v in G.split(U[wid], layout).items()}
        server.worker_data_queue.add_task((int(wid), int(n[wid]), d))
    for w in range(case["K"]):  # the initial broadcast of the previous model, once per worker
        server.worker_data_queue.get_result(consumer=w)
    res = server.worker_data_queue.get_result(consumer=0)
    flat = np.concatenate([res[nm].reshape(-1).cpu().numpy() for nm, _ in layout])
    assert same_bits(flat, z[f"{k}_full"])


def _union(Ud, n, subsets, P=None):
    from distributed_learning_simulator_amd import _native
    from distributed_learning_simulator_amd.aggregation import union_batch
    P = P or Ud.shape[1]
    t = union_batch(subsets, {i: int(n[i]) for i in range(len(n))}, dev)
    assert t is not None
    out = torch.full((len(subsets), P), float("nan"), device=dev)
    _native.subset_fedavg_union(Ud, *t, P, out)
    return out


@pytest.mark.parametrize("S", [1, 9, 17, 64])
def test_subset_union_bit_exact(S):
    """dls_subset_fedavg_union_f32 (every client row read once per batch) vs the
    reference op order, per coalition: rows in arbitrary order, > 64 clients
    (two chained launches), a ragged last tile, special values that send some
    tiles down the slow path (zeros, denormals, huge, inf, nan), and both
    division methods (a coalition total that fails the two-constant proof)."""
    K, P = 70, 4096 * 3 + 12
    g = torch.Generator().manual_seed(S)
    U = (torch.randn(K, P, generator=g) * 0.05).numpy()
    U[3, :8] = [0.0, -0.0, 1e-40, -1e-39, 3e38, np.inf, np.nan, 1e-45]
    U[:, 600:604] = 0.0  # a column of zeros in every client: -0 / +0 sums
    U[7, 5000] = -0.0
    n = [int(x) for x in torch.randint(1, 1001, (K,), generator=g)]
    perm = torch.randperm(K, generator=g).tolist()  # worker -> row
    subsets = []
    for s in range(S):
        k = int(torch.randint(1, K + 1, (1,), generator=g))
        members = sorted(torch.randperm(K, generator=g)[:k].tolist())
        subsets.append([perm[w] for w in members])
    subsets[0] = [perm[w] for w in range(K)]
    if S > 1:  # a divisor for which the two-constant quotient is not exact: Markstein
        n[5] = 11735695
        subsets[1] = [perm[5]]
    got = _union(torch.from_numpy(U).to(dev), n, subsets).cpu().numpy()
    for s, sub in enumerate(subsets):
        assert same_bits(got[s], _c.fedavg_ref(U, n, sub)), s


def test_subset_union_through_shapley_store():
    """ClientUpdateStore.subset_models takes the union kernel for sorted coalitions."""
    from distributed_learning_simulator_amd import _native
    from distributed_learning_simulator_amd.aggregation import ClientUpdateStore
    from distributed_learning_simulator_amd.layout import ParameterLayout
    calls = []
    orig = _native.subset_fedavg_union

    def spy(*a, **k):
        calls.append(1)
        return orig(*a, **k)

    lay = ParameterLayout([("w", (33, 31)), ("b", (5,))])
    st = ClientUpdateStore(lay, dev, capacity=12)
    g = torch.Generator().manual_seed(7)
    rows = [st.acquire() for _ in range(12)]
    for r in rows:
        st.write(r, {"w": torch.randn(33, 31, generator=g), "b": torch.randn(5, generator=g)})
    n = {r: 50 + 13 * r for r in rows}
    subs = [[rows[i] for i in sorted(torch.randperm(12, generator=g)[:1 + s % 12].tolist())]
            for s in range(70)]  # 70 coalitions: two union launches (64 + 6)
    _native.subset_fedavg_union = spy
    try:
        out = st.subset_models(subs, n).cpu().numpy()
    finally:
        _native.subset_fedavg_union = orig
    assert len(calls) == 2
    U = st.U.cpu().numpy()
    nn = [n.get(i, 1) for i in range(U.shape[0])]
    for s, sub in enumerate(subs):
        assert same_bits(out[s], _c.fedavg_ref(U, nn, sub)), s


def test_config5_scale_subset_kernels_resnet18():
    """BASELINE config 5 at its stated scale: 50 clients x full ResNet-18, S = 50
    GTG-like coalitions (sorted prefixes of random permutations).  Both exact
    kernels (union and per-coalition) bit-exact vs the oracle on 64Ki sampled
    parameters of every coalition; the fp32 MFMA GEMM normwise <= 1e-6 vs fp64."""
    from distributed_learning_simulator_amd import _native
    from distributed_learning_simulator_amd.layout import ParameterLayout
    from distributed_learning_simulator_amd.model_shapes import resnet18_cifar
    lay = ParameterLayout(resnet18_cifar())
    K, S, P = 50, 50, lay.P
    g = torch.Generator(device=dev).manual_seed(20250131)
    Ud = torch.empty((K, P), device=dev).normal_(generator=g).mul_(0.05)
    gc = torch.Generator().manual_seed(5)
    n = [int(x) for x in torch.randint(100, 1001, (K,), generator=gc)]
    subsets = []
    for s in range(S):
        perm = torch.randperm(K, generator=gc).tolist()
        subsets.append(sorted(perm[: 1 + (s * 7) % K]))
    cols = torch.sort(torch.randperm(lay.numel, generator=gc)[:1 << 16]).values
    cols_d = cols.to(dev)
    Uc = Ud[:, cols_d].cpu().numpy()
    # union kernel (the Shapley servers' default)
    got = _union(Ud, n, subsets)[:, cols_d].cpu().numpy()
    for s, sub in enumerate(subsets):
        assert same_bits(got[s], _c.fedavg_ref(Uc, n, sub)), ("union", s)
    # per-coalition kernel (dls_subset_fedavg_f32)
    off, rows, w, tot = [0], [], [], []
    for sub in subsets:
        rows += sub
        w += [n[r] for r in sub]
        tot.append(float(sum(n[r] for r in sub)))
        off.append(len(rows))
    out = torch.empty((S, P), device=dev)
    _native.subset_fedavg(Ud, torch.tensor(off, dtype=torch.int32, device=dev),
                          torch.tensor(rows, dtype=torch.int32, device=dev),
                          torch.tensor(w, dtype=torch.float32, device=dev),
                          torch.tensor(tot, dtype=torch.float32, device=dev), P, out)
    got = out[:, cols_d].cpu().numpy()
    for s, sub in enumerate(subsets):
        assert same_bits(got[s], _c.fedavg_ref(Uc, n, sub)), ("per-coalition", s)
    # MFMA contraction
    C = torch.zeros((S, K), dtype=torch.float64)
    for s, sub in enumerate(subsets):
        for r in sub:
            C[s, r] = n[r] / sum(n[i] for i in sub)
    _native.subset_gemm(C.float().to(dev), Ud, torch.arange(K, dtype=torch.int32, device=dev), P,
                        out)
    got = out[:, cols_d].cpu().double()
    ref = C @ torch.from_numpy(Uc).double()
    err = torch.linalg.norm(got - ref, dim=1) / torch.linalg.norm(ref, dim=1)
    assert float(err.max()) < 1e-6, float(err.max())
