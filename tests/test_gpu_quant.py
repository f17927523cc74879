"""GPU parity: fused dequant-FedAvg, min/max, qparams, quantize vs oracle / golden."""
import numpy as np
import pytest
import torch

from oracle import fedavg as ofed, quant as oquant
from tests import golden as G

pytestmark = pytest.mark.gpu

dev = torch.device("cuda")


def same_bits(a, b):
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    nan = np.isnan(a)
    return np.array_equal(nan, np.isnan(b)) and np.array_equal(
        a.view(np.uint32)[~nan], b.view(np.uint32)[~nan])


def assert_padding_zero(layout, full):
    """Every tile kind writes its tensor's 64-element row padding as zero (the
    re-quantization's per-tensor min / max spans it), whatever the buffer held."""
    f = full.cpu().numpy()
    ends = [o + m for o, m in zip(layout.offsets, layout.numels)]
    starts = layout.offsets[1:] + [layout.P]
    for a, b in zip(ends, starts):
        assert np.array_equal(f[a:b].view(np.uint32), np.zeros(b - a, np.uint32)), (a, b)


def golden_payloads():
    z = G.load("dequant.npz")
    case = G.meta(z)[0]
    layout, K = case["layout"], case["K"]
    payloads = []
    for i in range(K):
        d = {}
        for name, shape in layout:
            if name in case["qnames"]:
                d[name] = (torch.from_numpy(z[f"q{i}_{name}_int"].copy()),
                           torch.from_numpy(z[f"q{i}_{name}_scale"].copy()),
                           torch.from_numpy(z[f"q{i}_{name}_zp"].copy()))
            else:
                d[name] = torch.from_numpy(z[f"q{i}_{name}_f32"].copy())
        payloads.append(d)
    return z, case, payloads


def flat(views, layout):
    return np.concatenate([views[n].reshape(-1).cpu().numpy() for n, _ in layout])


def test_dequant_fedavg_golden_bit_exact():
    from distributed_learning_simulator_amd.quant_store import QuantizedClientStore
    z, case, payloads = golden_payloads()
    store = QuantizedClientStore(payloads[0], dev, capacity=2)  # forces a capacity grow
    rows = []
    for p in payloads:
        r = store.acquire()
        store.write(r, p)
        rows.append(r)
    for i, r in enumerate(rows):
        assert same_bits(flat(store.dequantize(r), case["layout"]), z[f"deq{i}"]), i
    out = store.fedavg(rows, [int(x) for x in z["n"]])
    assert same_bits(flat(store.layout.views(out), case["layout"]), z["agg"])


@pytest.mark.parametrize("granularity", ["model", "tensor"])
def test_fed_quant_server_round_golden(granularity):
    from distributed_learning_simulator_amd.servers.fed_quant_server import FedQuantServer
    z, case, payloads = golden_payloads()
    K = case["K"]
    server = FedQuantServer(tester=None, worker_number=K, synchronous=True,
                            granularity=granularity)
    for i, p in enumerate(payloads):
        server.worker_data_queue.add_task((i, int(z["n"][i]), p))
    for w in range(K):
        server.worker_data_queue.get_result(consumer=w)
    assert same_bits(flat(server.last_aggregate, case["layout"]), z["agg"])
    # the broadcast model is the re-quantized aggregate (this build's contract, D4)
    res = server.worker_data_queue.get_result(consumer=0)
    agg = z["agg"]
    if granularity == "tensor":
        q, sc, zp, deq = oquant.requantize_tensors(agg, case["layout"])
    else:  # one quantizer over concat_dict_values (ref servers/fed_quant_server.py:39)
        q, sc, zp, deq = oquant.requantize_model(agg)
        qg, scg, zpg = server.quantized_parameter
        assert np.array_equal(qg.cpu().numpy(), q)
        assert float(scg) == float(sc) and int(zpg) == zp
    assert same_bits(flat(res, case["layout"]), deq)


def test_fed_quant_model_granularity_resnet18_vs_torch_quantize_per_tensor():
    """the default re-quantization is the reference's one
    quantizer over the concatenated aggregate (servers/fed_quant_server.py:37-39).
    A full ResNet-18 round (2 int8 clients): the one-segment (scale, zero point)
    equal torch.ao's MinMaxObserver on the concatenated aggregate and the wire
    bytes equal torch.quantize_per_tensor's int_repr, in concat_dict_values order."""
    from distributed_learning_simulator_amd.model_shapes import resnet18_cifar
    from distributed_learning_simulator_amd.servers.fed_quant_server import FedQuantServer
    g = torch.Generator().manual_seed(44)
    payloads = []
    for k in range(2):
        p = {}
        for name, s in resnet18_cifar():
            if len(s) >= 2:
                p[name] = (torch.randint(-128, 128, s, generator=g, dtype=torch.int8),
                           torch.rand(s[0], generator=g, dtype=torch.float64) * 1e-3 + 1e-5,
                           torch.zeros(s[0], dtype=torch.int64))
            else:
                p[name] = torch.randn(s, generator=g) * 0.3
        payloads.append(p)
    server = FedQuantServer(tester=None, worker_number=2, synchronous=True)
    assert server.granularity == "model"
    for i, p in enumerate(payloads):
        server.worker_data_queue.add_task((i, 100 + 7 * i, p))
    for w in range(2):
        server.worker_data_queue.get_result(consumer=w)
    res = server.worker_data_queue.get_result(consumer=0)
    concat = torch.cat([v.reshape(-1) for v in server.last_aggregate.values()]).cpu()
    obs = torch.ao.quantization.MinMaxObserver(dtype=torch.quint8)
    obs(concat)
    sc_ref, zp_ref = obs.calculate_qparams()
    q, sc, zp = server.quantized_parameter
    assert q.numel() == concat.numel() and sc.numel() == 1 and zp.numel() == 1
    assert float(sc) == float(sc_ref) and int(zp) == int(zp_ref)
    qt = torch.quantize_per_tensor(concat, float(sc_ref), int(zp_ref), torch.quint8)
    assert torch.equal(q.cpu(), qt.int_repr())
    # the broadcast is the dequantized payload, tensor by tensor
    deq = torch.cat([v.reshape(-1) for v in res.values()]).cpu()
    assert torch.equal(deq, (qt.int_repr().float() - int(zp_ref)) * float(sc_ref))


@pytest.mark.parametrize("row_len", [1, 3, 15, 16, 17, 27, 576, 4099])
def test_dequant_fedavg_channel_shapes(row_len):
    """Channel rows shorter / longer than the 16-element lane chunk, int8 and uint8."""
    from distributed_learning_simulator_amd.quant_store import QuantizedClientStore
    g = torch.Generator().manual_seed(row_len)
    C = 37
    K = 3
    payloads, n = [], []
    for k in range(K):
        w8 = torch.randint(-128, 128, (C, row_len), generator=g, dtype=torch.int8)
        u8 = torch.randint(0, 256, (C + 1, row_len), generator=g, dtype=torch.uint8)
        payloads.append({
            "a": (w8, torch.rand(C, generator=g, dtype=torch.float64) * 1e-2,
                  torch.zeros(C, dtype=torch.int64)),
            "bias": torch.randn(C, generator=g),
            "b": (u8, torch.rand(C + 1, generator=g, dtype=torch.float64) * 1e-3,
                  torch.randint(0, 256, (C + 1,), generator=g)),
        })
        n.append(int(torch.randint(1, 1000, (1,), generator=g)))
    store = QuantizedClientStore(payloads[0], dev, capacity=K)
    rows = []
    for p in payloads:
        r = store.acquire()
        store.write(r, p)
        rows.append(r)
    full = torch.full((store.layout.P,), float("nan"), device=dev)  # stale memory
    out = store.layout.views(store.fedavg(rows, n, out=full))
    assert_padding_zero(store.layout, full)
    layout = [("a", (C, row_len)), ("bias", (C,)), ("b", (C + 1, row_len))]
    clients = [{k: (tuple(t.numpy() for t in v) if isinstance(v, tuple) else v.numpy())
                for k, v in p.items()} for p in payloads]
    ref = oquant.dequant_fedavg(clients, n, list(range(K)), layout)
    assert same_bits(flat(out, layout), ref)


def test_segment_minmax_qparams_quantize_vs_torch_formula():
    from distributed_learning_simulator_amd import _native
    z = G.load("quantize.npz")
    x = torch.from_numpy(z["pt_x"]).to(dev)
    total = x.numel()
    seg = torch.tensor([0, total], dtype=torch.int64, device=dev)
    scale = torch.tensor([float(z["pt_scale"])], dtype=torch.float32, device=dev)
    zp = torch.tensor([int(z["pt_zp"])], dtype=torch.int32, device=dev)
    q = torch.empty(total, dtype=torch.uint8, device=dev)
    _native.quantize_u8(x, seg, total, scale, zp, q)
    assert np.array_equal(q.cpu().numpy(), z["pt_q"])
    xt = torch.from_numpy(z["tie_x"]).to(dev)
    qt = torch.empty(xt.numel(), dtype=torch.uint8, device=dev)
    _native.quantize_u8(xt, torch.tensor([0, xt.numel()], dtype=torch.int64, device=dev),
                        xt.numel(), torch.tensor([0.0625], device=dev),
                        torch.tensor([10], dtype=torch.int32, device=dev), qt)
    assert np.array_equal(qt.cpu().numpy(), z["tie_q"])


def test_segment_minmax_many_segments():
    from distributed_learning_simulator_amd import _native
    g = torch.Generator().manual_seed(11)
    sizes = [1, 7, 64, 8191, 8192, 8193, 100000, 3, 20000]
    x = torch.randn(sum(sizes), generator=g)
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    seg = torch.from_numpy(off).to(dev)
    mins = torch.empty(len(sizes), device=dev)
    maxs = torch.empty(len(sizes), device=dev)
    _native.segment_minmax(x.to(dev), seg, int(off[-1]), mins, maxs)
    for s in range(len(sizes)):
        part = x[off[s]:off[s + 1]]
        assert float(mins[s]) == float(part.min()) and float(maxs[s]) == float(part.max())
    scale = torch.empty(len(sizes), device=dev)
    zp = torch.empty(len(sizes), dtype=torch.int32, device=dev)
    _native.qparams_minmax(mins, maxs, scale, zp)
    for s in range(len(sizes)):
        sc, z0 = oquant.minmax_qparams(float(mins[s]), float(maxs[s]))
        assert float(scale[s]) == float(sc) and int(zp[s]) == z0
    q = torch.empty(x.numel(), dtype=torch.uint8, device=dev)
    deq = torch.empty(x.numel(), device=dev)
    _native.quantize_u8(x.to(dev), seg, int(off[-1]), scale, zp, q, deq)
    for s in range(len(sizes)):
        sl = slice(off[s], off[s + 1])
        sc, z0 = oquant.minmax_qparams(float(mins[s]), float(maxs[s]))
        qr = oquant.quantize_affine(x[sl].numpy(), sc, z0)
        assert np.array_equal(q[sl].cpu().numpy(), qr)
        assert same_bits(deq[sl].cpu().numpy(), oquant.dequant_affine(qr, sc, z0))


def test_stochastic_quantize_unbiased():
    """Stochastic rounding (parity unpinned): E[deq] == x within sampling error."""
    from distributed_learning_simulator_amd import _native
    x = torch.full((1 << 20,), 0.3, device=dev)
    seg = torch.tensor([0, x.numel()], dtype=torch.int64, device=dev)
    scale = torch.tensor([0.25], device=dev)
    zp = torch.tensor([0], dtype=torch.int32, device=dev)
    q = torch.empty(x.numel(), dtype=torch.uint8, device=dev)
    deq = torch.empty_like(x)
    _native.quantize_u8(x, seg, x.numel(), scale, zp, q, deq, stochastic=True, seed=1234)
    vals = set(np.unique(q.cpu().numpy()).tolist())
    assert vals == {1, 2}
    assert abs(float(deq.mean()) - 0.3) < 1e-3


@pytest.mark.parametrize("K,L", [(1, 2500), (63, 2500), (64, 2500), (65, 2500), (130, 2500),
                                 (65, 11264), (3, 6144), (17, 3072), (9, 5120), (64, 1024),
                                 (130, 4160)])
def test_dequant_fedavg_chunked_clients_one_channel(K, L):
    """K across the kernels' 64-client chunks; long channel rows (one-channel
    tiles: 1 KiB tiles from the tensor start for L = 2500 / 4160, channel-aligned
    tiles of 4, 3, 2 and 1 KiB slices for the other L), int8 symmetric, uint8 with
    zero points for which fl(zp*s) is and is not exact, and a channel whose scale
    forces the IEEE-division path."""
    from distributed_learning_simulator_amd.quant_store import QuantizedClientStore
    g = torch.Generator().manual_seed(K * 7 + L)
    C = 5
    payloads, n = [], []
    for k in range(K):
        s8 = torch.rand(C, generator=g, dtype=torch.float64) * 1e-2 + 1e-4
        s8[3] = 3e30  # fl(deq * n) beyond the fast-division range
        su = torch.rand(C, generator=g, dtype=torch.float64) * 1e-3 + 1e-5
        su[0] = 0.0078125  # power of two: fl(zp * s) exact for every zp
        payloads.append({
            "a": (torch.randint(-128, 128, (C, L), generator=g, dtype=torch.int8), s8,
                  torch.zeros(C, dtype=torch.int64)),
            "b": (torch.randint(0, 256, (C, L), generator=g, dtype=torch.uint8), su,
                  torch.randint(0, 256, (C,), generator=g)),
            "bias": torch.randn(C, generator=g),
        })
        n.append(int(torch.randint(1, 1000, (1,), generator=g)))
    store = QuantizedClientStore(payloads[0], dev, capacity=K)
    rows = []
    for p in payloads:
        r = store.acquire()
        store.write(r, p)
        rows.append(r)
    assert sum(store.nfast) > 0
    if L % 1024 == 0 or L in (5120, 11264):
        assert store.nfast[4 - -(-min(L, 4096) // 1024)] > 0  # the widest slice group is used
    order = list(torch.randperm(K, generator=g).tolist())
    out = store.layout.views(store.fedavg([rows[i] for i in order], [n[i] for i in order]))
    layout = [("a", (C, L)), ("b", (C, L)), ("bias", (C,))]
    clients = [{k: (tuple(t.numpy() for t in v) if isinstance(v, tuple) else v.numpy())
                for k, v in p.items()} for p in payloads]
    ref = oquant.dequant_fedavg(clients, n, order, layout)
    assert same_bits(flat(out, layout), ref)


@pytest.mark.parametrize("total,two", [(11735695, 0), (55123, 1), (1 << 20, 1)])
def test_dequant_fedavg_division_methods(total, two):
    """The bulk kernels divide by fl32(N) with the two-constant method when the
    host's exhaustive check proves it exact for N, else with Markstein's
    correction: both bit-exact vs the oracle (N = 11,735,695 fails the check,
    55,123 passes it, 2^20 has yl = 0)."""
    import ctypes
    from distributed_learning_simulator_amd import _native
    from distributed_learning_simulator_amd.quant_store import QuantizedClientStore
    assert _native.lib().dls_two_constant_division(ctypes.c_float(total)) == two
    g = torch.Generator().manual_seed(total)
    C, L, K = 4, 4096, 3
    n = [total // 3, total // 3, total - 2 * (total // 3)]
    payloads = []
    for k in range(K):
        payloads.append({
            "a": (torch.randint(-128, 128, (C, L), generator=g, dtype=torch.int8),
                  torch.rand(C, generator=g, dtype=torch.float64) * 1e-2 + 1e-4,
                  torch.zeros(C, dtype=torch.int64)),
            "bias": torch.randn(C, generator=g),
        })
    store = QuantizedClientStore(payloads[0], dev, capacity=K)
    rows = []
    for p in payloads:
        r = store.acquire()
        store.write(r, p)
        rows.append(r)
    assert store.nfast[0] == C
    out = store.layout.views(store.fedavg(rows, n))
    layout = [("a", (C, L)), ("bias", (C,))]
    clients = [{k: (tuple(t.numpy() for t in v) if isinstance(v, tuple) else v.numpy())
                for k, v in p.items()} for p in payloads]
    ref = oquant.dequant_fedavg(clients, n, list(range(K)), layout)
    assert same_bits(flat(out, layout), ref)


def _full_model_store(shapes, K, seed):
    """K synthetic int8 payloads of a full model in a device store, filled the
    way bench.py fills it: raw int8 bytes, per-channel symmetric scales (zero
    point 0, the torch QAT default), fp32 1-d tensors."""
    from distributed_learning_simulator_amd.quant_store import QuantizedClientStore
    template = {}
    for name, s in shapes:
        if len(s) >= 2:
            template[name] = (torch.zeros(s, dtype=torch.int8),
                              torch.ones(s[0], dtype=torch.float64),
                              torch.zeros(s[0], dtype=torch.int64))
        else:
            template[name] = torch.zeros(s)
    st = QuantizedClientStore(template, dev, capacity=K)
    g = torch.Generator(device=dev).manual_seed(seed)
    st.Q.random_(0, 256, generator=g)  # raw int8 bytes
    st.F.normal_(generator=g)
    st.sz[..., 0].uniform_(1e-4, 1e-2, generator=g)
    st.sz[..., 1].zero_()  # symmetric int8 (torch QAT default)
    return st


def _check_sampled_channels(st, shapes, out, n, order, gc, extra_channels=None):
    """Every output element of three channels per int tensor (first, last, one
    random, plus ``extra_channels[name]``) and of every fp32 tensor, bit-exact vs
    the oracle run on those channels alone in the same client order."""
    import math
    K = st.capacity
    ql = st.qlayout
    clients = [dict() for _ in range(K)]
    layout, got = [], []
    for i, (name, s) in enumerate(shapes):
        if ql.kinds[i]:
            C, rl, src, cb = ql.channels[i], ql.row_len[i], ql.src[i], ql.chan_base[i]
            cs = sorted({0, C - 1, int(torch.randint(0, C, (1,), generator=gc))}
                        | set((extra_channels or {}).get(name, ())))
            q = torch.stack([st.Q[:, src + c * rl:src + (c + 1) * rl] for c in cs], 1)
            q = q.cpu().numpy().view(np.int8)  # [K, len(cs), rl]
            sc = st.sz[[cb + c for c in cs], :, 0].t().cpu().numpy().astype(np.float64)
            zp = st.sz[[cb + c for c in cs], :, 1].t().cpu().numpy().astype(np.int64)
            for k in range(K):
                clients[k][name] = (q[k], sc[k], zp[k])
            layout.append((name, (len(cs), rl)))
            got.append(out[name].reshape(C, rl)[cs].reshape(-1).cpu().numpy())
        else:
            m = math.prod(s)
            f = st.F[:, ql.src[i]:ql.src[i] + m].cpu().numpy()
            for k in range(K):
                clients[k][name] = f[k]
            layout.append((name, tuple(s)))
            got.append(out[name].reshape(-1).cpu().numpy())
    ref = oquant.dequant_fedavg(clients, n, order, layout)
    assert same_bits(np.concatenate(got), ref)


def test_dequant_fedavg_full_resnet18_k1000_sampled_channels():
    """The north-star instance bench.py times (fed_quant_k1000): 1000 clients x
    ResNet-18 int8 (11.2 GB in HBM) through the production tile table — every
    tile group the store builds (multi-channel lane tiles, fp32 tiles, the small
    int tiles of the 27-element first-conv rows), all 16 of the kernels'
    64-client chunks (15 full + one of 40), one client whose scale leaves the
    fast-division range on one channel of every int tensor (the per-client IEEE
    fallback of the lane and small-int kernels), clients in a shuffled reference order.  Sampled channels of
    every int tensor (including the fallback channel) and every fp32 tensor are
    bit-exact vs the oracle (ref servers/fed_quant_server.py:25-33 +
    servers/fed_server.py:44-66)."""
    from distributed_learning_simulator_amd.model_shapes import resnet18_cifar
    K = 1000
    shapes = resnet18_cifar()
    st = _full_model_store(shapes, K, seed=18)
    nf = st.nfast
    assert sum(nf[4:8]) > 0 and nf[8] > 0 and nf[9] > 0, nf  # lane, fp32, small int groups
    ql = st.qlayout
    gc = torch.Generator().manual_seed(18)
    bad_row = 613  # this client's channel 5 of every int tensor takes the IEEE path
    extra = {}
    for i, (name, s) in enumerate(shapes):
        if ql.kinds[i]:
            c = min(5, ql.channels[i] - 1)
            st.sz[ql.chan_base[i] + c, bad_row, 0] = 3e30
            extra[name] = (c,)
    n = torch.randint(100, 1001, (K,), generator=gc).tolist()
    order = torch.randperm(K, generator=gc).tolist()
    exact = st.fedavg(order, [n[r] for r in order])
    out = st.layout.views(exact)
    torch.cuda.synchronize()
    _check_sampled_channels(st, shapes, out, n, order, gc, extra)
    # the FMA mode (dls_dequant_fedavg_mode, DLS_FEDAVG_FMA) on the same 1000
    # clients: within the north-star FedAvg tolerance of the bit-exact aggregate
    # (normwise 1e-6), every tensor (the IEEE-fallback channel included)
    from distributed_learning_simulator_amd import _native
    fma = st.fedavg(order, [n[r] for r in order], mode=_native.FEDAVG_FMA)
    for name, v in st.layout.views(fma).items():
        e = out[name].double()
        err = float((v.double() - e).norm() / e.norm())
        assert err <= 1e-6, (name, err)
    assert not torch.equal(fma.view(torch.int32), exact.view(torch.int32))  # a different rounding


def test_dequant_fedavg_full_vgg16_sampled_channels():
    """BASELINE config 4 at full size: 100 clients x VGG-16 (13.8 GB of int8 in
    HBM, 138,357,544 parameters) through the production tile table.  Every
    output element of three channels per int tensor (first, last, one random:
    one-channel 4 KiB / 1 KiB tiles and the general kernel's conv rows) and of
    every fp32 tensor is checked bit-exactly against the oracle run on those
    channels alone, clients in a shuffled reference order."""
    from distributed_learning_simulator_amd.model_shapes import vgg16
    K = 100
    shapes = vgg16()
    st = _full_model_store(shapes, K, seed=4)
    gc = torch.Generator().manual_seed(4)
    n = torch.randint(100, 1001, (K,), generator=gc).tolist()
    order = torch.randperm(K, generator=gc).tolist()
    out = st.layout.views(st.fedavg(order, [n[r] for r in order]))
    torch.cuda.synchronize()
    _check_sampled_channels(st, shapes, out, n, order, gc)
    _check_fma_vs_exact(st, shapes, out, n, order, gc,
                        sampled=("classifier.0.weight", "classifier.3.weight", "classifier.6.weight"))


def _check_fma_vs_exact(st, shapes, exact, n, order, gc, sampled=()):
    """The FMA mode (dls_dequant_fedavg_mode DLS_FEDAVG_FMA) through the tile table
    bench.py times (store.table(FEDAVG_FMA)) vs the bit-exact aggregate: normwise
    <= 1e-6 per tensor (the north-star FedAvg tolerance); on three channel rows of
    each ``sampled`` tensor (first, last, one random: VGG-16's fc1 rows are 25,088
    elements, its one-channel FMA tiles) normwise <= 1e-6 per row and every element
    within 1e-6 of its magnitude sum sum_k (n_k / N) |q_k - zp_k| s_k (fp64 from the
    int8 payloads)."""
    from distributed_learning_simulator_amd import _native
    tiles, ntiles, nfast = st.table(_native.FEDAVG_FMA)
    assert tiles is st.tiles_fma and ntiles == st.ntiles_fma  # the bench's table
    fma = st.layout.views(st.fedavg(order, [n[r] for r in order], mode=_native.FEDAVG_FMA))
    for name, v in fma.items():
        e = exact[name].double()
        err = float((v.double() - e).norm() / e.norm())
        assert err <= 1e-6, (name, err)
    ql = st.qlayout
    names = [nm for nm, _ in shapes]
    w = torch.tensor(n, dtype=torch.float64, device=dev) / float(sum(n))  # row k holds client k
    for name in sampled:
        i = names.index(name)
        C, rl, src, cb = ql.channels[i], ql.row_len[i], ql.src[i], ql.chan_base[i]
        cs = sorted({0, C - 1, int(torch.randint(0, C, (1,), generator=gc))})
        for c in cs:
            q = st.Q[:, src + c * rl:src + (c + 1) * rl].view(torch.int8).double()  # [K, rl]
            sc = st.sz[cb + c, :, 0].double()[:, None]
            zp = st.sz[cb + c, :, 1].double()[:, None]
            mag = (w[:, None] * (q - zp).abs() * sc).sum(0)
            e = exact[name].reshape(C, rl)[c].double()
            d = (fma[name].reshape(C, rl)[c].double() - e).abs()
            assert float(d.norm() / e.norm()) <= 1e-6, (name, c)
            assert bool((d <= 1e-6 * mag).all()), (name, c, float((d / mag).max()))


def test_int8_symmetric_per_channel_quantize_golden():
    """The fed_quant worker's device path (workers/fed_quant_worker.py): int8
    (qmin = -128) per-channel quantize vs torch.quantize_per_channel's ints in
    quantize.npz (pc_*), and symmetric qparams vs torch.ao's per-channel
    symmetric MinMax observer (fp32 scale, zero point 0)."""
    from distributed_learning_simulator_amd import _native
    from distributed_learning_simulator_amd.workers.fed_quant_worker import \
        quantize_per_channel_symmetric
    z = G.load("quantize.npz")
    x = torch.from_numpy(z["pc_x"].copy())
    C = x.shape[0]
    row = x[0].numel()
    seg = (torch.arange(C + 1, dtype=torch.int64) * row).to(dev)
    scale = torch.from_numpy(z["pc_scale"].astype(np.float32)).to(dev)
    zp = torch.zeros(C, dtype=torch.int32, device=dev)
    q = torch.empty(x.numel(), dtype=torch.int8, device=dev)
    deq = torch.empty(x.numel(), device=dev)
    _native.quantize(x.reshape(-1).to(dev), seg, x.numel(), scale, zp, q, deq, qmin=-128, qmax=127)
    assert np.array_equal(q.cpu().numpy().reshape(z["pc_q"].shape), z["pc_q"])
    ref_deq = (z["pc_q"].astype(np.float32) * z["pc_scale"].astype(np.float32)[:, None, None])
    assert same_bits(deq.cpu().numpy(), ref_deq.reshape(-1))
    # the worker's whole chain: segment min/max -> symmetric qparams -> quantize
    obs = torch.ao.quantization.PerChannelMinMaxObserver(
        ch_axis=0, dtype=torch.qint8, qscheme=torch.per_channel_symmetric)
    obs(x)
    sc_ref, zp_ref = obs.calculate_qparams()
    qw, sc, zpw = quantize_per_channel_symmetric(x.to(dev))
    assert np.array_equal(sc.cpu().numpy(), sc_ref.float().numpy())
    assert np.array_equal(zpw.cpu().numpy(), zp_ref.int().numpy())
    qt = torch.quantize_per_channel(x, sc_ref.double(), zp_ref, 0, torch.qint8)
    assert np.array_equal(qw.cpu().numpy(), qt.int_repr().numpy())


def test_segment_minmax_ignores_nan():
    """NaNs are ignored (dls_hip.h) on both the bulk and the segment-boundary path;
    an all-NaN segment keeps the identities (+inf, -inf)."""
    from distributed_learning_simulator_amd import _native
    sizes = [5, 8190, 3, 9000, 1, 2]
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    g = torch.Generator().manual_seed(3)
    x = torch.rand(int(off[-1]), generator=g) + 0.5  # all positive
    x[torch.from_numpy(off[:4] + 1)] = float("nan")  # one NaN in each of the first 4 segments
    x[8185:8194] = float("nan")  # segment 1, across the 8192-element block boundary
    x[int(off[5]):] = float("nan")  # the last segment is all NaN
    mins = torch.empty(len(sizes), device=dev)
    maxs = torch.empty(len(sizes), device=dev)
    _native.segment_minmax(x.to(dev), torch.from_numpy(off).to(dev), int(off[-1]), mins, maxs)
    for s in range(len(sizes) - 1):
        part = x[off[s]:off[s + 1]]
        part = part[~torch.isnan(part)]
        assert float(mins[s]) == float(part.min()) and float(maxs[s]) == float(part.max()), s
    assert float(mins[-1]) == float("inf") and float(maxs[-1]) == float("-inf")


@pytest.mark.parametrize("K", [1, 70])
def test_dequant_fedavg_lane_tiles_resnet_shapes(K):
    """Multi-channel (lane) tiles: ResNet-like conv / fc weights whose channel rows
    are multiples of 16 (576, 1152, 32, 512), int8 symmetric and uint8 with zero
    points, K across the 64-client chunk, one client with a scale beyond the
    fast-division range (the per-client fallback); bit-exact vs the oracle."""
    from distributed_learning_simulator_amd.quant_store import QuantizedClientStore
    g = torch.Generator().manual_seed(K + 17)
    shapes = {"conv1": (5, 3, 3, 3), "l1": (8, 64, 3, 3), "l2": (4, 128, 3, 3),
              "sc": (3, 32, 1, 1), "fc": (10, 512)}
    payloads, n = [], []
    for k in range(K):
        p = {}
        for name, s in shapes.items():
            C = s[0]
            if name == "l2":  # uint8 with zero points
                p[name] = (torch.randint(0, 256, s, generator=g, dtype=torch.uint8),
                           torch.rand(C, generator=g, dtype=torch.float64) * 1e-3 + 1e-5,
                           torch.randint(0, 256, (C,), generator=g))
            else:
                sc = torch.rand(C, generator=g, dtype=torch.float64) * 1e-2 + 1e-4
                if k == K // 2 and name == "l1":
                    sc[2] = 3e30  # this client takes the fallback
                p[name] = (torch.randint(-128, 128, s, generator=g, dtype=torch.int8), sc,
                           torch.zeros(C, dtype=torch.int64))
            p[name + ".bias"] = torch.randn(C, generator=g)
        payloads.append(p)
        n.append(int(torch.randint(1, 1000, (1,), generator=g)))
    store = QuantizedClientStore(payloads[0], dev, capacity=K)
    assert sum(store.nfast[4:]) > 0  # lane tiles are used
    rows = []
    for p in payloads:
        r = store.acquire()
        store.write(r, p)
        rows.append(r)
    order = list(torch.randperm(K, generator=g).tolist())
    layout = [(k, tuple(v[0].shape) if isinstance(v, tuple) else tuple(v.shape))
              for k, v in payloads[0].items()]
    clients = [{k: (tuple(t.numpy() for t in v) if isinstance(v, tuple) else v.numpy())
                for k, v in p.items()} for p in payloads]
    ref = oquant.dequant_fedavg(clients, n, order, layout)
    from distributed_learning_simulator_amd import _native
    for mode in (_native.FEDAVG_EXACT, _native.FEDAVG_FMA):
        full = torch.full((store.layout.P,), float("nan"), device=dev)
        out = store.layout.views(store.fedavg([rows[i] for i in order], [n[i] for i in order],
                                              out=full, mode=mode))
        assert_padding_zero(store.layout, full)
        if mode == _native.FEDAVG_EXACT:
            assert same_bits(flat(out, layout), ref)
            continue
        # FMA mode: the int tensors on the grouped kernels take fma(q - z, c, acc)
        # with one constant per (client, channel), zero points included (the uint8
        # "l2"); the fp32 biases and the rows-of-27 conv (small-tile kernel) stay exact
        off = 0
        for name, shape in layout:
            m = int(np.prod(shape))
            got, want = out[name].reshape(-1).cpu().numpy(), ref[off:off + m]
            off += m
            if name == "conv1" or name.endswith(".bias"):
                assert same_bits(got, want), name
            else:
                err = np.linalg.norm(got.astype(np.float64) - want) / np.linalg.norm(want)
                assert err <= 1e-6, (name, err)


@pytest.mark.parametrize("lane_tile", ["adaptive", 4096])
def test_dequant_fedavg_exact_wide_lane_tiles(monkeypatch, lane_tile):
    """the EXACT mode on lane tiles of 2-4 KiB (k_dequant_lanes<4|3|2>,
    reachable through the ABI with any caller table): the adaptive widths and a
    fixed 4096-element table, with a client whose scale leaves the fast-division
    range (the per-client fallback) and a tile over more than 4 channels (rows of
    16: the per-client gather path); bit-exact vs the oracle, K across two
    64-client chunks."""
    from distributed_learning_simulator_amd import _native, quant_store as qs
    from distributed_learning_simulator_amd.quant_store import QTILE_DTYPE, QuantizedClientStore
    monkeypatch.setattr(qs, "LANE_TILE", lane_tile)
    K = 70
    g = torch.Generator().manual_seed(41)
    shapes = {"l1": (8, 64, 3, 3), "l2": (16, 128, 3, 3), "l3": (6, 256, 3, 3),
              "pw16": (64, 16, 1, 1), "fc": (10, 512)}
    payloads, n = [], []
    for k in range(K):
        p = {}
        for name, s_ in shapes.items():
            C = s_[0]
            if name == "l2":  # uint8 with zero points
                p[name] = (torch.randint(0, 256, s_, generator=g, dtype=torch.uint8),
                           torch.rand(C, generator=g, dtype=torch.float64) * 1e-3 + 1e-5,
                           torch.randint(0, 256, (C,), generator=g))
            else:
                sc = torch.rand(C, generator=g, dtype=torch.float64) * 1e-2 + 1e-4
                if k == K // 2 and name in ("l1", "pw16"):
                    sc[2] = 3e30  # this client takes the fallback
                p[name] = (torch.randint(-128, 128, s_, generator=g, dtype=torch.int8), sc,
                           torch.zeros(C, dtype=torch.int64))
        payloads.append(p)
        n.append(int(torch.randint(1, 1000, (1,), generator=g)))
    store = QuantizedClientStore(payloads[0], dev, capacity=K)
    t = store.tiles.cpu().numpy().view(QTILE_DTYPE)
    assert sum(store.nfast[4:7]) > 0  # 2-4 KiB lane tiles in the EXACT table
    lanes = t[sum(store.nfast[:4]):sum(store.nfast[:8])]
    span = (lanes["row_pos"] + lanes["len"] - 1) // lanes["row_len"] + 1
    if lane_tile == 4096:
        assert span.max() > 4  # the per-client gather path
    rows = []
    for p in payloads:
        r = store.acquire()
        store.write(r, p)
        rows.append(r)
    order = list(torch.randperm(K, generator=g).tolist())
    layout = [(k, tuple(v[0].shape)) for k, v in payloads[0].items()]
    clients = [{k: tuple(t_.numpy() for t_ in v) for k, v in p.items()} for p in payloads]
    ref = oquant.dequant_fedavg(clients, n, order, layout)
    full = torch.full((store.layout.P,), float("nan"), device=dev)
    out = store.layout.views(store.fedavg([rows[i] for i in order], [n[i] for i in order],
                                          out=full, mode=_native.FEDAVG_EXACT))
    assert_padding_zero(store.layout, full)
    assert same_bits(flat(out, layout), ref)


def test_dequant_fedavg_fma_lane_tiles_multipass(monkeypatch):
    """FMA-mode lane tiles over more channels than the kernel's staged table (4):
    1 KiB lane tiles on rows of 16, 48 and 64 elements (up to 64 channels per
    tile, walked in passes of 4 channels while the other lanes read the table's
    zero row), int8 symmetric and uint8 with zero points, K across two 64-client
    chunks; every tensor within the north-star 1e-6 normwise of the exact
    oracle.  The adaptive table never builds such tiles (it picks widths of at
    most 4 rows); a caller's fixed-width table may."""
    from distributed_learning_simulator_amd import _native, quant_store as qs
    from distributed_learning_simulator_amd.quant_store import QTILE_DTYPE, QuantizedClientStore
    monkeypatch.setattr(qs, "LANE_TILE_FMA", 1024)
    K = 70
    g = torch.Generator().manual_seed(29)
    shapes = {"pw16": (64, 16, 1, 1), "pw48": (40, 48, 1, 1), "pw64": (32, 64, 1, 1)}
    payloads, n = [], []
    for _ in range(K):
        p = {}
        for name, s in shapes.items():
            C = s[0]
            if name == "pw48":  # uint8 with zero points
                p[name] = (torch.randint(0, 256, s, generator=g, dtype=torch.uint8),
                           torch.rand(C, generator=g, dtype=torch.float64) * 1e-3 + 1e-5,
                           torch.randint(0, 256, (C,), generator=g))
            else:
                p[name] = (torch.randint(-128, 128, s, generator=g, dtype=torch.int8),
                           torch.rand(C, generator=g, dtype=torch.float64) * 1e-2 + 1e-4,
                           torch.zeros(C, dtype=torch.int64))
        payloads.append(p)
        n.append(int(torch.randint(1, 1000, (1,), generator=g)))
    store = QuantizedClientStore(payloads[0], dev, capacity=K)
    t = store.tiles_fma.cpu().numpy().view(QTILE_DTYPE)
    lanes = t[sum(store.nfast_fma[:4]):sum(store.nfast_fma[:8])]
    span = (lanes["row_pos"] + lanes["len"] - 1) // lanes["row_len"] + 1
    assert len(lanes) > 0 and span.max() > 4  # multi-pass tiles are used
    rows = []
    for p in payloads:
        r = store.acquire()
        store.write(r, p)
        rows.append(r)
    order = list(torch.randperm(K, generator=g).tolist())
    layout = [(k, tuple(v[0].shape)) for k, v in payloads[0].items()]
    clients = [{k: tuple(t.numpy() for t in v) for k, v in p.items()} for p in payloads]
    ref = oquant.dequant_fedavg(clients, n, order, layout)
    full = torch.full((store.layout.P,), float("nan"), device=dev)
    out = store.layout.views(store.fedavg([rows[i] for i in order], [n[i] for i in order],
                                          out=full, mode=_native.FEDAVG_FMA))
    assert_padding_zero(store.layout, full)
    off = 0
    for name, shape in layout:
        m = int(np.prod(shape))
        got, want = out[name].reshape(-1).cpu().numpy(), ref[off:off + m]
        off += m
        err = np.linalg.norm(got.astype(np.float64) - want) / np.linalg.norm(want)
        assert err <= 1e-6, (name, err)


def test_qat_weight_fake_quant_ste():
    """The fed_quant worker's quantization-aware training (ref
    workers/fed_quant_worker.py:19-20): conv / linear weights enter the forward
    pass as fl(q * scale) with torch's per-channel symmetric int8 qparams of the
    current weights, the gradient reaches the fp32 Parameter unchanged (STE), and
    the Parameter itself is restored after every forward.  The absent library's
    QAT details are not reproduced (parity unpinned); the fake-quantized weight
    is pinned bit-exact to torch.quantize_per_channel's ints times the scale."""
    import torch.nn.functional as F
    from distributed_learning_simulator_amd.workers.fed_quant_worker import (
        WeightFakeQuant, fake_quantize_per_channel_symmetric)
    g = torch.Generator().manual_seed(7)
    conv = torch.nn.Conv2d(3, 8, 3)
    lin = torch.nn.Linear(8 * 6 * 6, 10)
    model = torch.nn.Sequential(conv, torch.nn.ReLU(), torch.nn.Flatten(), lin).to(dev)
    for w in (conv.weight, lin.weight):
        obs = torch.ao.quantization.PerChannelMinMaxObserver(
            ch_axis=0, dtype=torch.qint8, qscheme=torch.per_channel_symmetric)
        wc = w.detach().cpu()
        obs(wc)
        sc, zp = obs.calculate_qparams()
        qi = torch.quantize_per_channel(wc, sc.double(), zp, 0, torch.qint8).int_repr().float()
        ref = qi * sc.float().view(-1, *([1] * (wc.dim() - 1)))
        assert torch.equal(fake_quantize_per_channel_symmetric(w).cpu(), ref)
    x = torch.randn((4, 3, 8, 8), generator=g).to(dev)
    hooks = WeightFakeQuant(model)
    y = model(x)
    assert isinstance(conv.weight, torch.nn.Parameter) and isinstance(lin.weight, torch.nn.Parameter)
    y.square().sum().backward()
    # the same forward with the fake-quantized weights as leaves
    cw = fake_quantize_per_channel_symmetric(conv.weight).requires_grad_()
    lw = fake_quantize_per_channel_symmetric(lin.weight).requires_grad_()
    y2 = F.linear(F.relu(F.conv2d(x, cw, conv.bias)).flatten(1), lw, lin.bias)
    y2.square().sum().backward()
    assert torch.allclose(y, y2, rtol=0, atol=1e-6)
    assert torch.allclose(conv.weight.grad, cw.grad, rtol=1e-5, atol=1e-6)
    assert torch.allclose(lin.weight.grad, lw.grad, rtol=1e-5, atol=1e-6)
    # a forward that raises leaves the Parameters in place (the hooks
    # used to park them until the next forward)
    with pytest.raises(RuntimeError):
        model(torch.randn((4, 5, 8, 8), device=dev))  # wrong channel count
    names = dict(model.named_parameters())
    assert names["0.weight"] is conv.weight and names["3.weight"] is lin.weight
    assert all(isinstance(p, torch.nn.Parameter) and p.is_leaf for p in names.values())
    # a deep copy (Trainer.get_inferencer(copy_model=True)) fake-quantizes ITS own
    # weights, and the hooked model pickles
    import copy
    import pickle
    twin = copy.deepcopy(model)
    with torch.no_grad():
        twin[0].weight.mul_(2.0)
        cw2 = fake_quantize_per_channel_symmetric(twin[0].weight)
        y3 = twin(x)
        ref3 = F.linear(F.relu(F.conv2d(x, cw2, twin[0].bias)).flatten(1),
                        fake_quantize_per_channel_symmetric(twin[3].weight), twin[3].bias)
    assert torch.allclose(y3, ref3, rtol=0, atol=1e-5)
    assert twin[0].weight is dict(twin.named_parameters())["0.weight"]
    assert len(pickle.dumps(model.cpu())) > 0
    model.to(dev)
    hooks.remove()
    plain = F.linear(F.relu(F.conv2d(x, conv.weight, conv.bias)).flatten(1), lin.weight, lin.bias)
    assert torch.allclose(model(x), plain, rtol=0, atol=1e-6)


@pytest.mark.parametrize("mode_name", ["exact", "fma"])
def test_dequant_fedavg_column_chunks_cutting_lane_tiles(mode_name):
    """the sharded fed_quant pipeline reduces column chunks in order
    (QuantizedClientStore.fedavg(cols=...)), each sub-table keeping the tiles that
    START in its range, so a multi-channel lane tile cut by a chunk bound writes
    past it into the next chunk.  With bounds placed inside lane tiles (and one
    inside a one-channel tile), the chunks run in order equal the whole table bit
    for bit, in both modes."""
    from distributed_learning_simulator_amd import _native
    from distributed_learning_simulator_amd.quant_store import QTILE_DTYPE, QuantizedClientStore
    mode = {"exact": _native.FEDAVG_EXACT, "fma": _native.FEDAVG_FMA}[mode_name]
    g = torch.Generator().manual_seed(77)
    shapes = {"l1": (8, 64, 3, 3), "l2": (16, 128, 3, 3), "fc": (6, 4096), "pw": (32, 64, 1, 1)}
    K = 5
    payloads, n = [], []
    for _ in range(K):
        p = {}
        for name, s_ in shapes.items():
            p[name] = (torch.randint(-128, 128, s_, generator=g, dtype=torch.int8),
                       torch.rand(s_[0], generator=g, dtype=torch.float64) * 1e-2 + 1e-4,
                       torch.zeros(s_[0], dtype=torch.int64))
            p[name + ".bias"] = torch.randn(s_[0], generator=g)
        payloads.append(p)
        n.append(int(torch.randint(1, 1000, (1,), generator=g)))
    store = QuantizedClientStore(payloads[0], dev, capacity=K)
    rows = []
    for p in payloads:
        r = store.acquire()
        store.write(r, p)
        rows.append(r)
    P = store.layout.P
    whole = store.fedavg(rows, n, mode=mode, out=torch.full((P,), float("nan"), device=dev))
    tiles, ntiles, nfast = store.table(mode)
    t = tiles.cpu().numpy().view(QTILE_DTYPE)[:ntiles]
    lanes = t[sum(nfast[:4]):sum(nfast[:8])]
    wide = lanes[lanes["len"] >= 64]
    assert len(wide) >= 2
    one = t[:sum(nfast[:4])]  # one-channel tiles (the EXACT table's fc rows; FMA: none)
    cuts = {int(wide[0]["dst"]) + 16, int(wide[len(wide) // 2]["dst"]) + 48}
    if len(one):
        cuts.add(int(one[0]["dst"]) + 32)
    cuts = sorted(cuts)
    bounds = [0] + cuts + [P]
    out = torch.full((P,), float("nan"), device=dev)
    crossing = 0
    for c0, c1 in zip(bounds[:-1], bounds[1:]):
        sub, nsub, _ = store.table(mode, (c0, c1))
        st = sub.cpu().numpy().view(QTILE_DTYPE)[:nsub]
        crossing += int(((st["dst"] + st["len"]) > c1).sum())
        store.fedavg(rows, n, out=out, mode=mode, cols=(c0, c1))
    assert crossing >= len(cuts)  # every cut lies inside a tile of the chunk before it
    assert torch.equal(out.view(torch.int32), whole.view(torch.int32))
