#!/usr/bin/env python3
"""Same-process, interleaved A/B of the whole utility forward (ResNet18.forward_split,
10k CIFAR-shaped images in one forward) across libdls_hip.so variants
(tools/build_variants.py -> tools/_variants/libdls_<name>.so).  Each variant packs
its own operands (the variants may differ in the split layouts) and runs whole
forwards; rounds alternate the variants so that clock drift hits all of them.

    python tools/forward_ab.py base new [--images 10000] [--rounds 5] [--reps 3]
"""
import argparse
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from distributed_learning_simulator_amd import _native  # noqa: E402
from distributed_learning_simulator_amd.models import ResNet18  # noqa: E402
from tools.conv_ab import load  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--images", type=int, default=10000)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    libs = [load(os.path.join(ROOT, "tools", "_variants", f"libdls_{v}.so")) for v in a.variants]
    torch.manual_seed(0)
    model = ResNet18().to(dev).eval()
    with torch.no_grad():
        for m in model.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.running_mean.uniform_(-0.2, 0.2)
                m.running_var.uniform_(0.5, 2.0)
    X = torch.randn(a.images, 3, 32, 32, device=dev, generator=torch.Generator(device=dev).manual_seed(1))
    pks, ref = [], []
    with torch.no_grad():
        for L in libs:
            _native._lib = L
            pks.append(model.pack_split())
            ref.append(model.forward_split(X, pks[-1]))
    times = [[] for _ in libs]
    same = [True for _ in libs]
    with torch.no_grad():
        for _ in range(a.rounds):
            for vi, L in enumerate(libs):
                _native._lib = L
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.reps):
                    out = model.forward_split(X, pks[vi])
                torch.cuda.synchronize()
                times[vi].append((time.perf_counter() - t0) / a.reps)
                same[vi] &= torch.equal(out.view(torch.int32), ref[vi].view(torch.int32))
    base = statistics.median(times[0])
    for vi, v in enumerate(a.variants):
        med = statistics.median(times[vi])
        print(f"{v:10s} forward of {a.images} images: median {med * 1e3:.2f} ms ({(med / base - 1) * 100:+.1f} %), "
              f"min {min(times[vi]) * 1e3:.2f}  repeatable {same[vi]}  "
              f"max |logit - {a.variants[0]}'s| {float((ref[vi] - ref[0]).abs().max()):.2e}")


if __name__ == "__main__":
    main()
