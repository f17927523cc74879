#!/usr/bin/env python3
"""Deterministic-convolution probe (csrc/conv.hip) on the GPU box.

1. every ResNet-18 conv shape once: dls_conv_bn_act_split vs an fp64 torch
   reference of conv + eval batch norm (+ residual) + ReLU, error relative to the
   abs-value convolution;
2. ResNet-18 forward_split vs the module's forward (fp32, MIOpen): top-1
   agreement and logit error on --images synthetic images;
3. the time of a --images evaluation through forward_split (batch --batch),
   per-kernel times through rocprofv3 when run under it.

    python tools/conv_probe.py [--images 10000] [--batch 1000] [--reps 3]
"""
import argparse
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_learning_simulator_amd import _native  # noqa: E402
from distributed_learning_simulator_amd.models import ResNet18  # noqa: E402


def layer_check(dev, B=8):
    g = torch.Generator(device=dev).manual_seed(0)
    worst = 0.0
    for (cin, cout, k, stride, H, res) in [(3, 64, 3, 1, 32, False), (64, 64, 3, 1, 32, True),
                                      (64, 128, 3, 2, 32, False), (64, 128, 1, 2, 32, False),
                                      (128, 128, 3, 1, 16, True), (128, 256, 3, 2, 16, False),
                                      (256, 512, 3, 2, 8, False), (512, 512, 3, 1, 4, True)]:
        x = torch.randn(B, cin, H, H, device=dev, generator=g)
        w = torch.randn(cout, cin, k, k, device=dev, generator=g) / (cin * k * k) ** 0.5
        bn = torch.nn.BatchNorm2d(cout).to(dev).eval()
        bn.running_mean.normal_(0, 0.3, generator=g)
        bn.running_var.uniform_(0.5, 2.0, generator=g)
        bn.weight.data.uniform_(0.5, 1.5, generator=g)
        bn.bias.data.normal_(0, 0.2, generator=g)
        consts = torch.empty(4 * cout, device=dev)
        _native.bn_fold_exact(bn, consts)
        s, pad = stride, k // 2
        ho = (H + 2 * pad - k) // s + 1
        r = torch.randn(B, cout, ho, ho, device=dev, generator=g) if res else None
        rs = _native.conv_pack_input(r) if res else None
        if cin < 32:  # the stem: a 1x1 convolution over the im2col
            xs = _native.conv_pack_im2col(x, (k, k), s, pad)
            ws = _native.conv_pack_weights_im2col(w)
            kk, s, pad = (1, 1), 1, 0
        else:
            xs = _native.conv_pack_input(x)
            ws = _native.conv_pack_weights(w)
            kk = (k, k)
        ys = _native.conv_bn_act(xs, ws, kk, s, pad, consts, rs, relu=True)
        y = _native.split_to_f32(ys)
        xd, wd = x.double(), w.double()
        ref = F.conv2d(xd, wd, stride=stride, padding=k // 2)
        absr = F.conv2d(xd.abs(), wd.abs(), stride=stride, padding=k // 2)
        m, iv = bn.running_mean.double(), 1 / torch.sqrt(bn.running_var.double() + bn.eps)
        sc = (bn.weight.double() * iv)[None, :, None, None]
        ref = (ref - m[None, :, None, None]) * sc + bn.bias.double()[None, :, None, None]
        if res:
            ref = ref + r.double()
        ref = ref.clamp_min(0)
        den = (absr * sc.abs() + (m[None, :, None, None] * sc).abs() + bn.bias.double().abs()[None, :, None, None]
               + ref.abs() + (r.double().abs() if res else 0) + 1e-30)
        err = ((y.double() - ref).abs() / den).max().item()
        ys2 = _native.conv_bn_act(xs, ws, kk, s, pad, consts, rs, relu=True)
        same = torch.equal(ys, ys2)
        worst = max(worst, err)
        print(f"conv {cin:3d}->{cout:3d} k{k} s{stride} H{H:2d} res={int(res)}: max rel err {err:.3e} "
              f"repeat bit-identical {same}", flush=True)
    return worst


def model_check(dev, n, batch):
    torch.manual_seed(0)
    model = ResNet18().to(dev).eval()
    for m in model.modules():  # non-trivial running statistics
        if isinstance(m, torch.nn.BatchNorm2d):
            m.running_mean.normal_(0, 0.1)
            m.running_var.uniform_(0.5, 1.5)
    X = torch.randn(n, 3, 32, 32, device=dev)
    with torch.no_grad():
        pk = model.pack_split()
        ours = torch.cat([model.forward_split(X[i:i + batch], pk) for i in range(0, n, batch)])
        ref = torch.cat([model(X[i:i + batch]) for i in range(0, n, batch)])
    top2 = ref.topk(2, dim=1).values
    margin = (top2[:, 0] - top2[:, 1])
    scale = ref.abs().amax(dim=1)
    diff = (ours - ref).abs().amax(dim=1)
    mism = ours.argmax(1) != ref.argmax(1)
    near = margin <= 1e-3 * scale
    print(f"model: {n} images, top-1 mismatches {int(mism.sum())} (of which near-ties "
          f"{int((mism & near).sum())}), max |logit diff| / max|logit| "
          f"{(diff / scale).max().item():.3e}", flush=True)
    return model, X


def timing(model, X, batch, reps):
    with torch.no_grad():
        for _ in range(2):
            pk = model.pack_split()
            for i in range(0, X.shape[0], batch):
                model.forward_split(X[i:i + batch], pk)
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            pk = model.pack_split()
            for i in range(0, X.shape[0], batch):
                model.forward_split(X[i:i + batch], pk).argmax(1)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
    ms = sorted(ts)[len(ts) // 2] * 1e3
    print(f"eval {X.shape[0]} images batch {batch}: {ms:.1f} ms -> {1e3 / ms:.2f} evals/s "
          f"(all {[round(t * 1e3, 1) for t in ts]})", flush=True)


RESNET18_CONVS = [  # (cin, cout, k, stride, H, residual, count per forward); the stem as 1x1 on its im2col
    (32, 64, 1, 1, 32, False, 1), (64, 64, 3, 1, 32, False, 2), (64, 64, 3, 1, 32, True, 2),
    (64, 128, 3, 2, 32, False, 1), (64, 128, 1, 2, 32, False, 1), (128, 128, 3, 1, 16, True, 2),
    (128, 128, 3, 1, 16, False, 1), (128, 256, 3, 2, 16, False, 1), (128, 256, 1, 2, 16, False, 1),
    (256, 256, 3, 1, 8, True, 2), (256, 256, 3, 1, 8, False, 1), (256, 512, 3, 2, 8, False, 1),
    (256, 512, 1, 2, 8, False, 1), (512, 512, 3, 1, 4, True, 2), (512, 512, 3, 1, 4, False, 1)]


def layer_times(dev, B=1000, n=20):
    """Per-conv-shape time of dls_conv_bn_act_split at batch B (n launches, HIP
    events), and the issued bf16 MFMA rate (3 products x 2 x padded MACs)."""
    tot = 0.0
    for (cin, cout, k, s, H, res, cnt) in RESNET18_CONVS:
        cp = _native.split_channels(cin)
        pad = k // 2
        ho = (H + 2 * pad - k) // s + 1
        x = torch.zeros(B, H, H, 2 * cp, dtype=torch.int16, device=dev)
        w = torch.zeros(cout, 2 * k * k * cp, dtype=torch.int16, device=dev)
        consts = torch.ones(4 * cout, device=dev)
        r = torch.zeros(B, ho, ho, 2 * cout, dtype=torch.int16, device=dev) if res else None
        y = torch.empty(B, ho, ho, 2 * cout, dtype=torch.int16, device=dev)
        for _ in range(3):
            _native.conv_bn_act(x, w, (k, k), s, pad, consts, r, True, out=y)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            _native.conv_bn_act(x, w, (k, k), s, pad, consts, r, True, out=y)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / n
        macs = B * ho * ho * cout * k * k * cp
        tot += ms * cnt
        print(f"layer {cin:3d}->{cout:3d} k{k} s{s} H{H:2d} res={int(res)} x{cnt}: {ms * 1e3:8.1f} us  "
              f"{6 * macs / ms / 1e9:7.1f} TFLOP/s bf16 issued", flush=True)
    # the fused-im2col stem (forward_split's first layer), replacing the 1x1 row above
    x = torch.randn(B, 3, 32, 32, device=dev)
    w = _native.conv_pack_weights_im2col(torch.randn(64, 3, 3, 3, device=dev))
    consts = torch.ones(4 * 64, device=dev)
    for _ in range(3):
        _native.conv_stem_bn_act(x, w, (3, 3), 1, 1, consts)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        _native.conv_stem_bn_act(x, w, (3, 3), 1, 1, consts)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    print(f"stem (fused im2col) 3-> 64 k3 s1 H32: {ms * 1e3:8.1f} us", flush=True)
    print(f"layers total per batch of {B}: {tot:.3f} ms (x10 = {10 * tot:.1f} ms per 10k-image eval; "
          f"the stem row as the 1x1 conv over its im2col)", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=10000)
    ap.add_argument("--batch", type=int, default=1000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--skip-check", action="store_true")
    ap.add_argument("--layers-only", action="store_true")
    ap.add_argument("--batches", default="", help="extra forward batch sizes to time, e.g. 2000,5000")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    # kernel variants are separate libraries (tools/build_variants.py, DLS_HIP_LIB):
    # the library picks its kernels from the shape alone
    for _ in range(1):
        print(f"== {os.environ.get('DLS_HIP_LIB', 'in-tree libdls_hip.so')}", flush=True)
        if not a.skip_check:
            layer_check(dev)
        layer_times(dev, a.batch)
        if not a.layers_only:
            model, X = model_check(dev, a.images, a.batch)
            timing(model, X, a.batch, a.reps)
            for b in [int(x) for x in a.batches.split(",") if x]:
                timing(model, X, b, a.reps)
            if a.batches:  # the logits do not depend on the batching
                with torch.no_grad():
                    pk = model.pack_split()
                    l1 = torch.cat([model.forward_split(X[i:i + a.batch], pk) for i in range(0, X.shape[0], a.batch)])
                    b = int(a.batches.split(",")[-1])
                    l2 = torch.cat([model.forward_split(X[i:i + b], pk) for i in range(0, X.shape[0], b)])
                print(f"logits batch {a.batch} vs {b} bit-identical: {torch.equal(l1, l2)}", flush=True)


if __name__ == "__main__":
    main()
