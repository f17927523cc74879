#!/usr/bin/env python3
"""Per-launch kernel times of one C-ABI call repeated back to back (HIP events
around each launch): is a kernel's time steady, ramping or bimodal?

    python tools/launch_series.py [--launches 300] [--what vote|fedavg1k|quant_r18]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from distributed_learning_simulator_amd import _native  # noqa: E402
from distributed_learning_simulator_amd.layout import ParameterLayout  # noqa: E402
from distributed_learning_simulator_amd.model_shapes import resnet18_cifar  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=300)
    ap.add_argument("--what", default="vote")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    P = ParameterLayout(resnet18_cifar()).P
    g = torch.Generator(device=dev).manual_seed(7)
    if args.what == "vote":
        K, W = 1000, _native.sign_words(P)
        planes = torch.randint(-2**62, 2**62, (K, W), generator=g, device=dev)
        planes[:, 1::2] &= ~planes[:, 0::2]
        so = torch.empty(P, device=dev)
        vp = torch.empty(W, dtype=torch.int64, device=dev)
        fn = lambda: _native.sign_vote(planes, None, K, P, so, vote_planes=vp)  # noqa: E731
    else:
        raise SystemExit("unknown --what")
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.launches)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    t = np.array([a.elapsed_time(b) for a, b in ev])
    q = np.percentile(t, [0, 10, 50, 90, 100])
    print(args.what, "percentiles 0/10/50/90/100 ms", np.round(q, 4).tolist(), flush=True)
    for i in range(0, args.launches, 20):
        print(f"  launches {i:4d}-{i + 19:4d}: median {np.median(t[i:i + 20]):.4f}  min {t[i:i + 20].min():.4f}")


if __name__ == "__main__":
    main()
