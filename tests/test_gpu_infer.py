"""GPU: the utility-evaluation inference path (get_metric,
servers/fed_server.py:26-32) with its hand-written eval batch norm.

* dls_bn_fold_f32 / dls_bn_act_nhwc_f32 against the same fp32 op sequence in
  torch (alpha = 1/sqrt(var+eps) * w, beta = b - mean * alpha, y = x*alpha + beta,
  + residual, ReLU): bit-exact, every flag combination, ragged sizes, C not a
  divisor of the grid (the per-iteration channel path), in place.
* dls_bn_fold_exact_f32 / dls_bn_act_exact_{nhwc,nchw}_f32 against torch's own eval
  BatchNorm2d on the GPU (MIOpen's inference kernel), + residual, ReLU: bit-exact.
* ResNet-18 forward_fused (the exact pass) vs torch's own eval forward: logits
  bit-identical with MIOpen's deterministic convolutions (its default kernels for
  the 512-channel layer vary run to run, the module's forward included); the
  Inferencer's accuracy and loss equal on both paths.
  Utility parity with the reference's tester is unpinned (its library is absent).
"""
import time

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
dev = torch.device("cuda", 0)


def _bn(C, g):
    bn = torch.nn.BatchNorm2d(C).to(dev).eval()
    with torch.no_grad():
        bn.weight.copy_(torch.rand(C, generator=g) + 0.5)
        bn.bias.copy_(torch.randn(C, generator=g) * 0.1)
        bn.running_mean.copy_(torch.randn(C, generator=g) * 0.2)
        bn.running_var.copy_(torch.rand(C, generator=g) + 0.1)
    return bn


def _ref_fold(bn):
    invstd = 1.0 / torch.sqrt(bn.running_var + bn.eps)
    a = invstd * bn.weight
    return a, bn.bias - bn.running_mean * a


@pytest.mark.parametrize("N,C,H,W", [(3, 64, 7, 5), (2, 96, 3, 3), (5, 512, 4, 4), (1, 12, 1, 1)])
@pytest.mark.parametrize("res,relu", [(False, True), (True, True), (False, False), (True, False)])
def test_bn_act_bit_exact(N, C, H, W, res, relu):
    from distributed_learning_simulator_amd import _native
    g = torch.Generator().manual_seed(N * C + H)
    bn = _bn(C, g)
    a = torch.empty(C, device=dev)
    b = torch.empty(C, device=dev)
    _native.bn_fold(bn, a, b)
    ra, rb = _ref_fold(bn)
    assert torch.equal(a.view(torch.int32), ra.detach().view(torch.int32))
    assert torch.equal(b.view(torch.int32), rb.detach().view(torch.int32))
    cl = torch.channels_last
    x = torch.randn(N, C, H, W, generator=g).to(dev).contiguous(memory_format=cl)
    x[0, 0, 0, 0] = float("nan")
    r = torch.randn(N, C, H, W, generator=g).to(dev).contiguous(memory_format=cl) if res else None
    y = _native.bn_act_nhwc(x, a, b, residual=r, relu=relu)
    ref = x * a[None, :, None, None] + b[None, :, None, None]
    if res:
        ref = ref + r
    if relu:
        ref = torch.relu(ref)
    assert y.is_contiguous(memory_format=cl)
    assert torch.isnan(y[0, 0, 0, 0])
    m = ~torch.isnan(ref)
    assert torch.equal(y[m].view(torch.int32), ref[m].view(torch.int32))
    y2 = _native.bn_act_nhwc(x.clone(memory_format=cl), a, b, residual=r, relu=relu, inplace=True)
    assert torch.equal(y2[m].view(torch.int32), ref[m].view(torch.int32))


def test_bn_act_rejects_nchw():
    from distributed_learning_simulator_amd import _native
    x = torch.randn(2, 8, 3, 3, device=dev)
    with pytest.raises(RuntimeError):
        _native.bn_act_nhwc(x, torch.ones(8, device=dev), torch.zeros(8, device=dev))


@pytest.mark.parametrize("N,C,H,W", [(64, 64, 32, 32), (16, 128, 16, 16), (7, 512, 4, 4),
                                     (3, 12, 5, 3), (2, 96, 3, 3)])
@pytest.mark.parametrize("res,relu", [(False, True), (True, True), (False, False)])
def test_bn_act_exact_matches_torch_eval(N, C, H, W, res, relu):
    """The exact pass = torch's eval BatchNorm2d (+ residual add, ReLU) bit for bit,
    channels_last fp32, NaN kept, in place."""
    from distributed_learning_simulator_amd import _native
    g = torch.Generator().manual_seed(N + C + H)
    bn = _bn(C, g)
    with torch.no_grad():
        bn.running_var[0] = 1e-3  # small variances too
    consts = torch.empty(4 * C, device=dev)
    _native.bn_fold_exact(bn, consts)
    cl = torch.channels_last
    x = (torch.randn(N, C, H, W, generator=g) * 3).to(dev).contiguous(memory_format=cl)
    x[0, 0, 0, 0] = float("nan")
    r = torch.randn(N, C, H, W, generator=g).to(dev).contiguous(memory_format=cl) if res else None
    with torch.no_grad():
        ref = bn(x)
        if res:
            ref = ref + r
        if relu:
            ref = torch.relu(ref)
    y = _native.bn_act_exact_nhwc(x, consts, residual=r, relu=relu)
    assert y.is_contiguous(memory_format=cl)
    assert torch.isnan(y[0, 0, 0, 0]) and torch.isnan(ref[0, 0, 0, 0])
    m = ~torch.isnan(ref)
    assert torch.equal(y[m].view(torch.int32), ref[m].view(torch.int32))
    y2 = _native.bn_act_exact_nhwc(x.clone(memory_format=cl), consts, residual=r, relu=relu,
                                   inplace=True)
    assert torch.equal(y2[m].view(torch.int32), ref[m].view(torch.int32))


@pytest.mark.parametrize("N,C,H,W", [(64, 64, 32, 32), (16, 128, 16, 16), (7, 512, 4, 4),
                                     (3, 12, 5, 4), (2, 96, 2, 6)])
@pytest.mark.parametrize("res,relu", [(False, True), (True, True), (False, False)])
def test_bn_act_exact_nchw_matches_torch_eval(N, C, H, W, res, relu):
    """The exact pass over NCHW-contiguous activations (dls_bn_act_exact_nchw_f32,
    the deterministic utility path's layout) = torch's eval BatchNorm2d (+ residual
    add, ReLU) bit for bit, NaN kept, in place; channel counts and planes that are
    and are not powers of two."""
    from distributed_learning_simulator_amd import _native
    g = torch.Generator().manual_seed(N + 3 * C + H)
    bn = _bn(C, g)
    with torch.no_grad():
        bn.running_var[0] = 1e-3
    consts = torch.empty(4 * C, device=dev)
    _native.bn_fold_exact(bn, consts)
    x = (torch.randn(N, C, H, W, generator=g) * 3).to(dev)
    x[0, 0, 0, 0] = float("nan")
    r = torch.randn(N, C, H, W, generator=g).to(dev) if res else None
    with torch.no_grad():
        ref = bn(x)
        if res:
            ref = ref + r
        if relu:
            ref = torch.relu(ref)
    y = _native.bn_act_exact(x, consts, residual=r, relu=relu)
    assert y.is_contiguous()
    assert torch.isnan(y[0, 0, 0, 0]) and torch.isnan(ref[0, 0, 0, 0])
    m = ~torch.isnan(ref)
    assert torch.equal(y[m].view(torch.int32), ref[m].view(torch.int32))
    y2 = _native.bn_act_exact_nchw(x.clone(), consts, residual=r, relu=relu, inplace=True)
    assert torch.equal(y2[m].view(torch.int32), ref[m].view(torch.int32))
    with pytest.raises(RuntimeError):  # a channels_last activation is not NCHW
        _native.bn_act_exact_nchw(x.contiguous(memory_format=torch.channels_last), consts)


@pytest.fixture
def deterministic_convs():
    """MIOpen's convolutions for ResNet-18's 512-channel layer pick a kernel whose
    result varies between two runs of the same input (tools/diag_fused.py: the
    module's own forward twice is not bit-identical); its deterministic mode makes
    the module's forward a function, so the fused path can be compared bit for bit."""
    old = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    yield
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = old


@pytest.mark.parametrize("fmt", ["nhwc", "nchw"])
def test_resnet18_fused_eval_matches_torch(deterministic_convs, fmt):
    from distributed_learning_simulator_amd.models import ResNet18, synthetic_classification
    from distributed_learning_simulator_amd.trainer import Inferencer
    torch.manual_seed(0)
    model = ResNet18().to(dev)
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for m in model.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.running_mean.copy_(torch.randn(m.num_features, generator=g) * 0.1)
                m.running_var.copy_(torch.rand(m.num_features, generator=g) + 0.5)
                m.weight.copy_(torch.rand(m.num_features, generator=g) + 0.5)
                m.bias.copy_(torch.randn(m.num_features, generator=g) * 0.1)
    X, y = synthetic_classification(600, (3, 32, 32), seed=3)
    mf = torch.channels_last if fmt == "nhwc" else torch.contiguous_format
    model.eval().to(memory_format=mf)
    xb = X.to(dev).contiguous(memory_format=mf)
    if fmt == "nhwc":  # MIOpen's deterministic NHWC convolutions are its naive kernels
        xb = xb[:64]
        y = y[:64]
        X = X[:64]
    with torch.no_grad():
        ref = model(xb)
        assert torch.equal(model(xb).view(torch.int32), ref.view(torch.int32))  # a function
        got = model.forward_fused(xb, model.fold_bn())
    assert torch.equal(got.view(torch.int32), ref.view(torch.int32))  # the same bits
    # the Inferencer takes the fused path on the GPU by default; fused_eval=False the
    # module's forward: the same accuracy and loss, and those of torch's eval
    # forward over the same batches (MIOpen may pick other algorithms for other
    # batch sizes)
    inf = Inferencer(model, (X, y), batch_size=256, device=dev, conv="miopen")
    assert inf.fused_eval is True and inf.deterministic  # the NCHW path
    loss, acc, _ = inf.inference()
    plain = Inferencer(model, (X, y), batch_size=256, device=dev, fused_eval=False, conv="miopen")
    loss0, acc0, _ = plain.inference()
    assert acc == acc0 and float(loss) == float(loss0)
    xq = X.to(dev)  # the Inferencer's deterministic layout: NCHW
    with torch.no_grad():
        pred = torch.cat([model(xq[i:i + 256]).argmax(1) for i in range(0, xq.shape[0], 256)])
    assert acc0 == int((pred.cpu() == y).sum()) / y.numel()  # the Inferencer's int / n
    assert np.isfinite(float(loss))


def test_utility_is_a_function_of_the_model():
    """VERDICT r03 item 1, for the MIOpen path (conv="miopen"; the default tester's
    own convolutions: tests/test_gpu_conv.py): bit-identical logits and the same
    accuracy / loss for the same model on repeated evaluations and on fresh
    Inferencers, at ResNet-18 x 10k CIFAR-shaped images (the config-5 utility), and
    torch's global flags as it found them.  And it stays fast: MIOpen's
    deterministic NHWC convolutions are naive kernels (19 s per evaluation,
    profiles/r04q_eval_det.txt), the NCHW path ~0.2 s."""
    from distributed_learning_simulator_amd.models import ResNet18, synthetic_classification
    from distributed_learning_simulator_amd.trainer import Inferencer
    torch.manual_seed(7)
    model = ResNet18().to(dev)
    X, y = synthetic_classification(10000, (3, 32, 32), seed=11)
    flags = (torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark)
    a = Inferencer(model, (X, y), device=dev, conv="miopen")
    assert a.deterministic and a.fused_eval
    la = a.logits()
    la2 = a.logits()
    loss_a, acc_a, _ = a.inference()
    assert (torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark) == flags
    b = Inferencer(model, (X, y), device=dev, conv="miopen")
    lb = b.logits()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    loss_b, acc_b, _ = b.inference()
    assert time.perf_counter() - t0 < 3.0  # not MIOpen's naive-kernel fallback
    assert a._fused_checked == (torch.contiguous_format, True)  # fused pass == bn(x) here
    assert torch.equal(la.view(torch.int32), la2.view(torch.int32))
    assert torch.equal(la.view(torch.int32), lb.view(torch.int32))
    assert acc_a == acc_b and float(loss_a) == float(loss_b)
    assert acc_a == int((la.argmax(1).cpu() == y).sum()) / y.numel()
    # the module's own forward under the same flags: the same bits
    plain = Inferencer(model, (X, y), device=dev, fused_eval=False, conv="miopen")
    assert torch.equal(plain.logits().view(torch.int32), la.view(torch.int32))


def test_inferencer_odd_plane_sizes():
    """ResNet-18's adaptive pooling takes any input size; a 28x28 input
    reaches layer3 as 7x7 planes (49 elements, not a multiple of 4), which the
    NCHW exact pass runs element-wise: the default Inferencer's logits equal the
    module's own forward, bit for bit."""
    from distributed_learning_simulator_amd import _native
    from distributed_learning_simulator_amd.models import ResNet18, synthetic_classification
    from distributed_learning_simulator_amd.trainer import Inferencer
    torch.manual_seed(3)
    model = ResNet18().to(dev)
    X, y = synthetic_classification(512, (3, 28, 28), seed=5)
    a = Inferencer(model, (X, y), device=dev, conv="miopen")
    la = a.logits()
    assert a._fused_checked == (torch.contiguous_format, True)
    plain = Inferencer(model, (X, y), device=dev, fused_eval=False, conv="miopen")
    assert torch.equal(plain.logits().view(torch.int32), la.view(torch.int32))
    # the kernel alone on odd planes, with a residual and ReLU, vs torch
    g = torch.Generator().manual_seed(1)
    bn = _bn(24, g)
    consts = torch.empty(4 * 24, device=dev)
    _native.bn_fold_exact(bn, consts)
    x = torch.randn(3, 24, 7, 5, generator=g).to(dev)
    r = torch.randn(3, 24, 7, 5, generator=g).to(dev)
    got = _native.bn_act_exact(x, consts, residual=r, relu=True)
    with torch.no_grad():
        ref = torch.relu(bn(x) + r)
    assert torch.equal(got.view(torch.int32), ref.view(torch.int32))
