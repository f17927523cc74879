#!/usr/bin/env python3
"""Per-layer time per image of dls_conv_bn_act_split (csrc/conv.hip) at several
batch sizes, on random operands (zero operands run at a higher clock,
MI355X_MICROARCH.md).  (Round 6 also timed per-stage sub-batch schedules of the
forward here — stem + layer1 on 256-1000-image sub-batches so their activations
stay in the Infinity Cache: all 1-5 % slower than whole-batch stages,
profiles/r06_conv_stage_probe.txt; the schedule was dropped.)

    python tools/conv_stage_probe.py --layers [--batches 1000,10000]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_learning_simulator_amd import _native  # noqa: E402
from tools.conv_probe import RESNET18_CONVS  # noqa: E402


def _time(fn, n):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def layer_sweep(dev, batches, n=20):
    g = torch.Generator(device=dev).manual_seed(0)
    tot = [0.0] * len(batches)
    for (cin, cout, k, s, H, res, cnt) in RESNET18_CONVS[1:]:
        pad = k // 2
        ho = (H + 2 * pad - k) // s + 1
        w = _native.conv_pack_weights(torch.randn(cout, cin, k, k, device=dev, generator=g) / (cin * k * k) ** 0.5)
        consts = torch.cat([torch.zeros(cout, device=dev), torch.ones(cout, device=dev),
                            torch.ones(cout, device=dev), torch.zeros(cout, device=dev)])
        row = []
        for bi, B in enumerate(batches):
            x = _native.conv_pack_input(torch.randn(B, cin, H, H, device=dev, generator=g).relu_())
            r = _native.conv_pack_input(torch.randn(B, cout, ho, ho, device=dev, generator=g)) if res else None
            y = torch.empty(B, ho, ho, 2 * cout, dtype=torch.int16, device=dev)
            ms = _time(lambda: _native.conv_bn_act(x, w, (k, k), s, pad, consts, r, True, out=y), n)
            row.append(f"B={B}: {ms * 1e3 / B * 1000:7.1f} us/1000img")
            tot[bi] += cnt * ms * 1e3 / B * 1000
            del x, r, y
        print(f"layer {cin:3d}->{cout:3d} k{k} s{s} H{H:2d} res={int(res)} x{cnt}: " + "  ".join(row), flush=True)
    row = []
    w = _native.conv_pack_weights_im2col(torch.randn(64, 3, 3, 3, device=dev, generator=g) / 27 ** 0.5)
    consts = torch.cat([torch.zeros(64, device=dev), torch.ones(128, device=dev), torch.zeros(64, device=dev)])
    for bi, B in enumerate(batches):
        x = torch.randn(B, 3, 32, 32, device=dev, generator=g)
        ms = _time(lambda: _native.conv_stem_bn_act(x, w, (3, 3), 1, 1, consts), n)
        row.append(f"B={B}: {ms * 1e3 / B * 1000:7.1f} us/1000img")
        tot[bi] += ms * 1e3 / B * 1000
    print("stem (fused im2col) 3-> 64 k3 s1 H32:  " + "  ".join(row), flush=True)
    print("total per 1000 images (every conv of the forward): " +
          "  ".join(f"B={B}: {t:7.1f} us" for B, t in zip(batches, tot)), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", action="store_true")
    ap.add_argument("--batches", default="250,500,1000,2500,10000")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    print(f"== {os.environ.get('DLS_HIP_LIB', 'in-tree libdls_hip.so')}", flush=True)
    if a.layers:
        layer_sweep(dev, [int(b) for b in a.batches.split(",")])


if __name__ == "__main__":
    main()
