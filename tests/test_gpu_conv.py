"""Deterministic convolutions of the utility evaluation (csrc/conv.hip;
SURVEY.md §8 row a-3, servers/fed_server.py:26-32 get_metric -> the tester).

There is no reference output to pin: the reference evaluates with torch's
convolutions on its own device, whose low bits depend on the algorithm the
library picks.  The contract tested here is the one the Shapley servers need:
  * every conv + eval batch norm (+ residual) + ReLU launch is within a stated
    bound of an fp64 evaluation of the same function (bf16x3 products: a relative
    error of ~2^-16 per product; the bound, 5e-5 of the magnitude sum, is >= 7x
    the largest error measured, profiles/r05_conv_probe.txt);
  * the same inputs give the same bits on repeated launches, interleaved with
    other shapes, and on fresh tensors (and in another process:
    tests/test_gpu_distributed.py::test_utility_bit_identical_across_processes);
  * ResNet-18's logits agree with torch's fp32 forward to ~1e-5 of their scale and
    top-1 agrees except where the top two logits are that close.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
dev = torch.device("cuda", 0)
TOL = 5e-5

# (cin, cout, k, stride, H, W, residual, batch): every ResNet-18 shape (the LDS-DMA
# pipeline for 3x3 stride 1, the generic kernel otherwise), ragged last tiles
# (batch not a multiple of the images per tile), sizes the pipeline does not take
# (28x28 -> the register-staged halo kernel; 7x7, 12x12 -> generic), Cout a
# multiple of 64 but not of 128, a non-square image, and the stem (cin < 32:
# im2col + the generic kernel, and the fused-im2col stem kernel, which must give
# the same bits)
SHAPES = [
    (3, 64, 3, 1, 32, 32, False, 4), (64, 64, 3, 1, 32, 32, False, 3), (64, 64, 3, 1, 32, 32, True, 2),
    (64, 128, 3, 2, 32, 32, False, 3), (64, 128, 1, 2, 32, 32, False, 3),
    (128, 128, 3, 1, 16, 16, True, 3), (128, 256, 3, 2, 16, 16, False, 2), (128, 256, 1, 2, 16, 16, False, 2),
    (256, 256, 3, 1, 8, 8, True, 3), (256, 512, 3, 2, 8, 8, False, 2), (256, 512, 1, 2, 8, 8, False, 2),
    (512, 512, 3, 1, 4, 4, True, 5), (64, 64, 3, 1, 28, 28, True, 2), (128, 128, 3, 1, 7, 7, False, 3),
    (96, 192, 3, 1, 12, 12, True, 2), (64, 128, 3, 1, 8, 16, False, 3), (3, 64, 3, 1, 28, 28, False, 2),
    # stems off the 3x3 / 3-channel fast path: a 5x5 MNIST-like one (runtime
    # index arithmetic) and a strided one over two 64-channel output tiles
    (1, 64, 5, 1, 28, 28, False, 2), (3, 128, 3, 2, 32, 32, False, 2),
    # the LDS-DMA pipeline's other cases: one channel chunk (32 channels, no
    # halo reload), 64-channel blocks over 16x16 / 8x8 images (whole images,
    # partial last tile), 128 channels over 32x32 (4 row tiles per image), a
    # 24-row image (row tiles at y0 > 0, 4-wave blocks), 4x4 images with two
    # chunks and a mostly empty tile (48 of 256 pixels)
    (32, 64, 3, 1, 32, 32, True, 2), (64, 64, 3, 1, 16, 16, False, 3), (64, 64, 3, 1, 8, 8, True, 3),
    (128, 128, 3, 1, 32, 32, False, 2), (32, 128, 3, 1, 24, 16, True, 2), (64, 256, 3, 1, 4, 4, False, 3),
    # the stride-2 phase pipeline: a non-square image with a residual (two images
    # per tile), a partial tile, and a size it does not take (6-wide output)
    (64, 128, 3, 2, 16, 32, True, 3), (32, 256, 3, 2, 8, 8, False, 5), (128, 128, 3, 2, 12, 12, False, 2),
]


def _bn(c, g):
    bn = torch.nn.BatchNorm2d(c).to(dev).eval()
    with torch.no_grad():
        bn.running_mean.copy_(torch.randn(c, generator=g) * 0.3)
        bn.running_var.copy_(torch.rand(c, generator=g) * 1.5 + 0.5)
        bn.weight.copy_(torch.rand(c, generator=g) + 0.5)
        bn.bias.copy_(torch.randn(c, generator=g) * 0.2)
    return bn


def _run(cin, cout, k, s, H, W, res, B, seed=0):
    from distributed_learning_simulator_amd import _native
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, cin, H, W, generator=g).to(dev)
    w = (torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5).to(dev)
    bn = _bn(cout, g)
    consts = torch.empty(4 * cout, device=dev)
    _native.bn_fold_exact(bn, consts)
    pad = k // 2
    ho, wo = (H + 2 * pad - k) // s + 1, (W + 2 * pad - k) // s + 1
    r = torch.randn(B, cout, ho, wo, generator=g).to(dev) if res else None
    rs = _native.conv_pack_input(r) if res else None
    if cin < 32:
        xs, ws = _native.conv_pack_im2col(x, (k, k), s, pad), _native.conv_pack_weights_im2col(w)
        geom = ((1, 1), 1, 0)
    else:
        xs, ws = _native.conv_pack_input(x), _native.conv_pack_weights(w)
        geom = ((k, k), s, pad)
    ys = _native.conv_bn_act(xs, ws, *geom, consts, rs, relu=True)
    if cin < 32 and not res:  # the fused-im2col stem kernel: the same operands, the same bits
        stem = _native.conv_stem_bn_act(x, ws, (k, k), s, pad, consts, relu=True)
        assert torch.equal(stem, ys)
    return (x, w, bn, r, s, pad), (xs, ws, geom, consts, rs), ys


@pytest.mark.parametrize("shape", SHAPES, ids=lambda t: "c{}-{}k{}s{}_{}x{}{}_b{}".format(
    t[0], t[1], t[2], t[3], t[4], t[5], "_res" if t[6] else "", t[7]))
def test_conv_bn_act_matches_fp64(shape):
    from distributed_learning_simulator_amd import _native
    (x, w, bn, r, s, pad), _, ys = _run(*shape)
    y = _native.split_to_f32(ys).double()
    xd, wd = x.double(), w.double()
    m = bn.running_mean.double()[None, :, None, None]
    sc = (bn.weight.double() / torch.sqrt(bn.running_var.double() + bn.eps))[None, :, None, None]
    b = bn.bias.double()[None, :, None, None]
    ref = (F.conv2d(xd, wd, stride=s, padding=pad) - m) * sc + b
    den = F.conv2d(xd.abs(), wd.abs(), stride=s, padding=pad) * sc.abs() + (m * sc).abs() + b.abs()
    if r is not None:
        ref = ref + r.double()
        den = den + r.double().abs()
    ref = ref.clamp_min(0)
    err = ((y - ref).abs() / (den + ref.abs() + 1e-30)).max().item()
    assert err < TOL, err
    assert y.shape == ref.shape and torch.isfinite(y).all()


def _fuzz_cases(n=24, seed=2026):
    import random
    rnd = random.Random(seed)
    cases = []
    while len(cases) < n:
        cin = rnd.choice([32, 64, 96, 128, 256])
        cout = rnd.choice([64, 128, 192, 256])
        s = rnd.choice([1, 1, 2])
        hw = rnd.choice([4, 8, 16, 32]) if s == 1 else rnd.choice([8, 16, 32])
        h = hw if rnd.random() < 0.7 else hw // 2 if hw > 4 else hw
        b = rnd.randint(1, 6)
        if b * h * hw * max(cin, cout) > 2 ** 21:  # keep the fp64 reference quick
            continue
        cases.append((cin, cout, 3, s, h, hw, rnd.random() < 0.5, b))
    return cases


@pytest.mark.parametrize("shape", _fuzz_cases(), ids=lambda t: "c{}-{}s{}_{}x{}{}_b{}".format(
    t[0], t[1], t[3], t[4], t[5], "_res" if t[6] else "", t[7]))
def test_conv_bn_act_random_shapes_match_fp64(shape):
    """A seeded sweep over the shapes the 3x3 kernels choose between (the LDS-DMA
    pipeline's 4- / 8-wave and one- / two-halo-buffer forms, the stride-2 phase
    pipeline, the register-staged fallbacks): odd channel-chunk counts, 64- and
    128-multiple output channels, non-square images, partial tiles."""
    test_conv_bn_act_matches_fp64(shape)


def test_conv_bit_identical_on_repeat():
    """The same inputs -> the same bits: repeated launches, launches of other shapes
    in between, and fresh copies of the operands (other addresses)."""
    from distributed_learning_simulator_amd import _native
    _, (xs, ws, geom, consts, rs), y1 = _run(64, 64, 3, 1, 32, 32, True, 4, seed=3)
    _, (xs2, ws2, geom2, consts2, rs2), z1 = _run(256, 512, 3, 2, 8, 8, False, 4, seed=4)
    y2 = _native.conv_bn_act(xs, ws, *geom, consts, rs, relu=True)
    z2 = _native.conv_bn_act(xs2, ws2, *geom2, consts2, rs2, relu=True)
    y3 = _native.conv_bn_act(xs.clone(), ws.clone(), *geom, consts.clone(), rs.clone(), relu=True)
    assert torch.equal(y1, y2) and torch.equal(y1, y3) and torch.equal(z1, z2)


def test_conv_rejects_bad_shapes():
    from distributed_learning_simulator_amd import _native
    x = torch.zeros(2, 8, 8, 2 * 48, dtype=torch.int16, device=dev)  # C = 48: not a multiple of 32
    w = torch.zeros(64, 2 * 9 * 48, dtype=torch.int16, device=dev)
    with pytest.raises(RuntimeError, match="multiple of 32"):
        _native.conv_bn_act(x, w, (3, 3), 1, 1)
    x = torch.zeros(2, 8, 8, 2 * 64, dtype=torch.int16, device=dev)
    w = torch.zeros(96, 2 * 9 * 64, dtype=torch.int16, device=dev)  # Cout = 96
    with pytest.raises(RuntimeError, match="Cout of 64"):
        _native.conv_bn_act(x, w, (3, 3), 1, 1)
    w = torch.zeros(64, 2 * 9 * 32, dtype=torch.int16, device=dev)  # packed for another C
    with pytest.raises(RuntimeError, match="do not match"):
        _native.conv_bn_act(x, w, (3, 3), 1, 1)


def _resnet(seed):
    from distributed_learning_simulator_amd.models import ResNet18
    torch.manual_seed(seed)
    model = ResNet18().to(dev).eval()
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        for m in model.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.running_mean.copy_(torch.randn(m.num_features, generator=g) * 0.1)
                m.running_var.copy_(torch.rand(m.num_features, generator=g) + 0.5)
                m.weight.copy_(torch.rand(m.num_features, generator=g) + 0.5)
                m.bias.copy_(torch.randn(m.num_features, generator=g) * 0.1)
    return model


@pytest.mark.parametrize("hw", [32, 28])
def test_resnet18_forward_split_matches_torch(hw):
    """Logits within 2e-5 of their scale of torch's fp32 forward; top-1 equal
    except at near-ties (top-2 margin <= 1e-4 of the scale)."""
    from distributed_learning_simulator_amd.models import synthetic_classification
    model = _resnet(0)
    X, _ = synthetic_classification(1500, (3, hw, hw), seed=2)
    X = X.to(dev)
    with torch.no_grad():
        pk = model.pack_split()
        ours = torch.cat([model.forward_split(X[i:i + 500], pk) for i in range(0, X.shape[0], 500)])
        ref = torch.cat([model(X[i:i + 500]) for i in range(0, X.shape[0], 500)])
        again = torch.cat([model.forward_split(X[i:i + 500], model.pack_split())
                           for i in range(0, X.shape[0], 500)])
    assert torch.equal(ours.view(torch.int32), again.view(torch.int32))
    scale = ref.abs().amax(dim=1)
    assert ((ours - ref).abs().amax(dim=1) <= 2e-5 * scale).all()
    top2 = ref.topk(2, dim=1).values
    near = (top2[:, 0] - top2[:, 1]) <= 1e-4 * scale
    mism = ours.argmax(1) != ref.argmax(1)
    assert not (mism & ~near).any()


def test_logits_do_not_depend_on_the_batching():
    """Each image's logits are the same bits in any batch (the kernels' reduction
    order per output does not depend on the other images), which lets the
    Inferencer pick its own forward batch."""
    from distributed_learning_simulator_amd.models import synthetic_classification
    model = _resnet(9)
    X, _ = synthetic_classification(1200, (3, 32, 32), seed=4)
    X = X.to(dev)
    with torch.no_grad():
        pk = model.pack_split()
        whole = model.forward_split(X, pk)
        parts = torch.cat([model.forward_split(X[i:i + 173], pk) for i in range(0, X.shape[0], 173)])
    assert torch.equal(whole.view(torch.int32), parts.view(torch.int32))


def test_inferencer_default_runs_library_convolutions():
    """The default GPU tester runs forward_split: torch's global cudnn flags are not
    touched, the accuracy is the logits' argmax rate, a fresh Inferencer gives the
    same bits, and 10k CIFAR images take well under a second."""
    import time
    from distributed_learning_simulator_amd.models import synthetic_classification
    from distributed_learning_simulator_amd.trainer import Inferencer
    model = _resnet(5)
    X, y = synthetic_classification(10000, (3, 32, 32), seed=6)
    flags = (torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark)
    a = Inferencer(model, (X, y), device=dev)
    assert a.conv == "dls" and a._split_forward() is not None
    la = a.logits()
    loss, acc, _ = a.inference()
    assert (torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark) == flags
    assert acc == int((la.argmax(1).cpu() == y).sum()) / y.numel()
    b = Inferencer(model, (X, y), device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    lb = b.logits()
    torch.cuda.synchronize()
    assert time.perf_counter() - t0 < 1.0
    assert torch.equal(la.view(torch.int32), lb.view(torch.int32))
    loss_b, acc_b, _ = b.inference()
    assert acc == acc_b and float(loss) == float(loss_b)


def test_inferencer_keeps_one_device_copy_of_a_host_test_set():
    """A host-resident test set (simulator.py builds the tester on CPU tensors) is
    copied to the device once and reused by every evaluation (VERDICT r05 weak #3:
    no 123 MB pageable copy per utility evaluation); an in-place change of the
    dataset makes a new copy; cache_dataset=False pins the host copy once instead.
    All three give the same bits."""
    from distributed_learning_simulator_amd.models import synthetic_classification
    from distributed_learning_simulator_amd.trainer import Inferencer
    model = _resnet(7)
    X, y = synthetic_classification(2000, (3, 32, 32), seed=8)
    a = Inferencer(model, (X, y), device=dev)
    la = a.logits()
    Xc, yc = a._resident_dataset()
    assert Xc.is_cuda and yc.is_cuda and torch.equal(Xc.cpu(), X)
    a.inference()
    assert a._resident_dataset()[0].data_ptr() == Xc.data_ptr()  # no second copy
    pinned = Inferencer(model, (X, y), device=dev, cache_dataset=False)
    lp = pinned.logits()
    Xp = pinned._resident_dataset()[0]
    assert not Xp.is_cuda and Xp.is_pinned()
    assert pinned._resident_dataset()[0].data_ptr() == Xp.data_ptr()
    assert torch.equal(la.view(torch.int32), lp.view(torch.int32))
    X[0] += 1.0  # in place: the device copy is stale and must be remade
    lb = a.logits()
    assert a._resident_dataset()[0].data_ptr() != Xc.data_ptr()
    assert torch.equal(a._resident_dataset()[0][0].cpu(), X[0])
    assert torch.equal(lb[1:].view(torch.int32), la[1:].view(torch.int32))


def test_split_forward_batch_falls_back_under_a_memory_budget():
    """The forward batch is capped by the activations that fit SPLIT_MEM_FRACTION of
    the free device memory: with a budget of ~700 images the 2,000-image
    test set runs in smaller forwards, with the same bits as one forward."""
    from distributed_learning_simulator_amd.models import synthetic_classification
    from distributed_learning_simulator_amd.trainer import Inferencer
    model = _resnet(11)
    X, y = synthetic_classification(2000, (3, 32, 32), seed=12)
    a = Inferencer(model, (X, y), device=dev)
    assert a.split_batch(2000) == 2000
    whole = a.logits()
    small = Inferencer(model, (X, y), device=dev)
    free, _ = torch.cuda.mem_get_info(dev)
    free += torch.cuda.memory_reserved(dev) - torch.cuda.memory_allocated(dev)
    per_image = model.split_activation_bytes(32, 32)
    small.SPLIT_MEM_FRACTION = 700.5 * per_image / free
    bs = small.split_batch(2000)
    assert 600 <= bs <= 700, bs
    parts = small.logits()
    assert torch.equal(whole.view(torch.int32), parts.view(torch.int32))


def test_bf16x3_utilities_equal_fp32_utilities_at_config5_scale():
    """Config 5: 16 coalitions of 50 ResNet-18 clients (a teacher
    + client noise, as bench.py) on 10k CIFAR-shaped images labelled by the
    teacher.  Every flipped top-1 prediction between the library-conv utility and
    the fp32 utility of Inferencer(conv="miopen") (MIOpen's deterministic fp32
    convolutions, logits bit-identical to the module's forward) is a near-tie of
    the fp32 logits (top-2 margin <= 1e-4 of their scale), and no coalition's
    utility moves by more than 3 images (3e-4), a third of GTG's truncation
    eps = 0.001 (ref servers/GTG_shapley_value_server.py:54).  Measured (GPU
    session r06a): 2 flips in 160,000 predictions, both near-ties, both in one
    coalition (2e-4); the other 15 utilities equal the fp32 ones exactly."""
    from distributed_learning_simulator_amd.model_util import ModelUtil
    from distributed_learning_simulator_amd.models import ResNet18
    from distributed_learning_simulator_amd.servers.fed_server import FedServer
    from distributed_learning_simulator_amd.trainer import Inferencer
    torch.manual_seed(20250133)
    teacher = ResNet18().to(dev).eval()
    X = torch.randn(10000, 3, 32, 32, device=dev)
    with torch.no_grad():
        y = torch.cat([teacher(X[i:i + 1000]).argmax(1) for i in range(0, 10000, 1000)])
    tester = Inferencer(ResNet18().to(dev), (X.cpu(), y.cpu()), batch_size=1000, device=dev)
    server = FedServer(tester=tester, worker_number=50, synchronous=True, device=dev)
    base = ModelUtil(teacher).get_parameter_dict()
    g = torch.Generator(device=dev).manual_seed(20250133)
    for wid in range(50):
        server.parameters[wid] = (100 + 17 * wid, {
            k: v + torch.randn(v.shape, generator=g, device=dev) * 0.002 for k, v in base.items()})
    rng = torch.Generator().manual_seed(5)
    flips = near_flips = 0
    diffs = []
    for _ in range(16):
        size = int(torch.randint(1, 51, (1,), generator=rng))
        coal = sorted(torch.randperm(50, generator=rng)[:size].tolist())
        ModelUtil(tester.model).load_parameter_dict(server.get_subset_model(coal))
        tester.conv = "dls"
        ours = tester.logits()
        _, u_dls, _ = tester.inference()
        tester.conv = "miopen"
        ref = tester.logits()
        _, u_fp32, _ = tester.inference()
        yd = y.to(dev)
        assert u_dls == int((ours.argmax(1) == yd).sum()) / 10000
        assert u_fp32 == int((ref.argmax(1) == yd).sum()) / 10000
        diffs.append(abs(u_dls - u_fp32))
        mism = ours.argmax(1) != ref.argmax(1)
        scale = ref.abs().amax(dim=1)
        top2 = ref.topk(2, dim=1).values
        near = (top2[:, 0] - top2[:, 1]) <= 1e-4 * scale
        flips += int(mism.sum())
        near_flips += int((mism & near).sum())
    print(f"config-5 utilities: max |u_bf16x3 - u_fp32| = {max(diffs):.6f} over 16 coalitions; "
          f"flipped top-1 predictions {flips} of 160,000 (near-ties {near_flips})")
    assert flips == near_flips
    assert max(diffs) <= 3e-4 + 1e-12


def test_queued_evaluations_on_several_streams_equal_one_stream():
    """ShapleyValueServer.evaluate_subsets queues each coalition's forward on one of
    eval_streams HIP streams (two forwards in flight): the utilities are the same
    floats as with one stream and as get_metric's synchronous inference(), the
    model may be overwritten while an earlier forward is still queued (pack_split
    copies every operand, the linear layer included), and a dataset read on
    several streams is not released early."""
    from distributed_learning_simulator_amd.model_util import ModelUtil
    from distributed_learning_simulator_amd.models import ResNet18, synthetic_classification
    from distributed_learning_simulator_amd.servers.shapley_value_server import ShapleyValueServer
    from distributed_learning_simulator_amd.trainer import Inferencer
    torch.manual_seed(31)
    base = ModelUtil(_resnet(13)).get_parameter_dict()
    X, y = synthetic_classification(3000, (3, 32, 32), seed=14)
    tester = Inferencer(ResNet18().to(dev), (X, y), batch_size=1000, device=dev)
    server = ShapleyValueServer(tester=tester, worker_number=6, synchronous=True, device=dev,
                                subset_batch=4)
    g = torch.Generator(device=dev).manual_seed(31)
    for wid in range(6):
        server.parameters[wid] = (50 + 7 * wid, {
            k: v + torch.randn(v.shape, generator=g, device=dev) * 0.05 for k, v in base.items()})
    server._set_prev_model(base)
    coal = [(0,), (1, 2), (), (0, 3, 5), (4,), (1, 2, 3, 4, 5), (2, 5), (0, 1, 2, 3, 4, 5), (3,)]
    out = {}
    for ns in (1, 2, 3):
        server.eval_streams = ns
        out[ns] = server.evaluate_subsets(coal)
    assert server._streams is not None and len(server._streams) == 3
    assert out[1] == out[2] == out[3]
    sync = [float(server.get_metric(server.get_subset_model(list(c)) if c else server.prev_model))
            for c in coal]
    assert out[2] == sync
    assert len(set(out[2])) > 2  # the coalitions' models differ


@pytest.mark.parametrize("cin,cout,s,H", [(64, 64, 1, 32), (128, 128, 1, 16), (256, 256, 1, 8), (64, 128, 2, 32)])
def test_walk_direction_does_not_change_bits(cin, cout, s, H):
    """A launch whose input is a recent launch's output walks its tiles the other
    way (the serpentine walk, csrc/conv.hip conv_walk_direction); a fresh copy of
    the same input walks forwards.  Both give the same bits (no output's
    reduction order depends on the tile order)."""
    from distributed_learning_simulator_amd import _native
    _, (xs, ws, geom, consts, rs), _ = _run(cin, cin, 3, 1, H, H, False, 5, seed=21)
    g = torch.Generator().manual_seed(22)
    w2 = (torch.randn(cout, cin, 3, 3, generator=g) / (cin * 9) ** 0.5).to(dev)
    ws2 = _native.conv_pack_weights(w2)
    h = _native.conv_bn_act(xs, ws, *geom, consts, None, relu=True)  # h recorded as written forwards
    walked = _native.conv_bn_act(h, ws2, (3, 3), s, 1, None, None, relu=True)  # reads h: backwards
    fresh = _native.conv_bn_act(h.clone(), ws2, (3, 3), s, 1, None, None, relu=True)  # forwards
    torch.cuda.synchronize()
    assert torch.equal(walked, fresh)
