#!/usr/bin/env python3
"""Same-process, interleaved A/B timing of the utility convolutions
(dls_conv_bn_act_split, dls_conv_stem_bn_act_f32) across libdls_hip.so variants
(tools/build_variants.py -> tools/_variants/libdls_<name>.so), every ResNet-18
shape at one batch, on random operands (cdna_hip_programming.md §5.4 rules 24-25).

    python tools/conv_ab.py base prio comajor [--batch 10000] [--rounds 5] [--launches 5]

Prints per shape the median time per 1000 images of each variant, whether every
variant's output is bit-identical to the first's, whether every variant's
untimed call of each round reproduced its own first output, and the per-forward total
(each shape weighted by its count in ResNet-18).
"""
import argparse
import ctypes
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from distributed_learning_simulator_amd import _native  # noqa: E402
from tools.conv_probe import RESNET18_CONVS  # noqa: E402


def load(path):
    L = ctypes.CDLL(path)
    for name, (args, res) in _native.SIGNATURES.items():
        f = getattr(L, name, None)
        if f is not None:
            f.argtypes, f.restype = args, res
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--batch", type=int, default=10000)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--launches", type=int, default=5)
    ap.add_argument("--shapes", default="", help="indices into RESNET18_CONVS (default all) + 'stem'")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    libs = [load(os.path.join(ROOT, "tools", "_variants", f"libdls_{v}.so")) for v in a.variants]
    g = torch.Generator(device=dev).manual_seed(0)
    B = a.batch
    cases = []
    sel = a.shapes.split(",") if a.shapes else [str(i) for i in range(1, len(RESNET18_CONVS))] + ["stem"]
    for key in sel:
        if key == "stem":
            x = torch.randn(B, 3, 32, 32, device=dev, generator=g)
            w32 = torch.randn(64, 3, 3, 3, device=dev, generator=g) / 27 ** 0.5
            ws = []
            for L in libs:  # each variant packs its own weights (its layout)
                _native._lib = L
                ws.append(_native.conv_pack_weights_im2col(w32))
            consts = torch.cat([torch.zeros(64, device=dev), torch.ones(128, device=dev), torch.zeros(64, device=dev)])
            cases.append(("stem (fused im2col) 3-> 64 k3 s1 H32", 1,
                          lambda vi, x=x, ws=ws, c=consts: _native.conv_stem_bn_act(x, ws[vi], (3, 3), 1, 1, c)))
            continue
        cin, cout, k, s, H, res, cnt = RESNET18_CONVS[int(key)]
        pad = k // 2
        ho = (H + 2 * pad - k) // s + 1
        w32 = torch.randn(cout, cin, k, k, device=dev, generator=g) / (cin * k * k) ** 0.5
        ws = []
        for L in libs:
            _native._lib = L
            ws.append(_native.conv_pack_weights(w32))
        _native._lib = libs[0]
        consts = torch.cat([torch.randn(cout, device=dev, generator=g) * 0.1, torch.ones(cout, device=dev),
                            torch.ones(cout, device=dev), torch.zeros(cout, device=dev)])
        x = _native.conv_pack_input(torch.randn(B, cin, H, H, device=dev, generator=g).relu_())
        r = _native.conv_pack_input(torch.randn(B, cout, ho, ho, device=dev, generator=g)) if res else None
        cases.append((f"{cin:3d}->{cout:3d} k{k} s{s} H{H:2d} res={int(res)} x{cnt}", cnt,
                      lambda vi, x=x, ws=ws, c=consts, r=r, k=k, s=s, pad=pad:
                      _native.conv_bn_act(x, ws[vi], (k, k), s, pad, c, r, True)))
    tot = [0.0] * len(libs)
    print(f"batch {B}, {a.rounds} rounds x {a.launches} launches, variants {a.variants}", flush=True)
    for name, cnt, fn in cases:
        outs = []
        for vi, L in enumerate(libs):
            _native._lib = L
            outs.append(fn(vi))
        same = all(torch.equal(o, outs[0]) for o in outs[1:])
        ts = [[] for _ in libs]
        stable = True  # every variant's every untimed call reproduces its first output (a race screen)
        for _ in range(a.rounds):
            for vi, L in enumerate(libs):
                _native._lib = L
                stable &= torch.equal(fn(vi), outs[vi])
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.launches):
                    fn(vi)
                e1.record()
                torch.cuda.synchronize()
                ts[vi].append(e0.elapsed_time(e1) / a.launches * 1e3 * 1000 / B)
        med = [statistics.median(t) for t in ts]
        for vi in range(len(libs)):
            tot[vi] += cnt * med[vi]
        cells = "  ".join(f"{v}={m:7.1f}" + (f" ({(m / med[0] - 1) * 100:+5.1f}%)" if vi else "")
                          for vi, (v, m) in enumerate(zip(a.variants, med)))
        del outs
        print(f"{name}: {cells}  bits-equal {same}  repeatable {stable}", flush=True)
    cells = "  ".join(f"{v}={t:7.1f}" + (f" ({(t / tot[0] - 1) * 100:+5.1f}%)" if vi else "")
                      for vi, (v, t) in enumerate(zip(a.variants, tot)))
    print(f"TOTAL us per 1000 images (every conv of one forward): {cells}", flush=True)


if __name__ == "__main__":
    main()
