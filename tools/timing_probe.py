#!/usr/bin/env python3
"""Probe: per-launch HIP-event timing vs one event pair around N launches (FedAvg K=100)."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from distributed_learning_simulator_amd import _native  # noqa: E402
from distributed_learning_simulator_amd.layout import ParameterLayout  # noqa: E402
from distributed_learning_simulator_amd.model_shapes import resnet18_cifar  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    P = ParameterLayout(resnet18_cifar()).P
    K = 100
    g = torch.Generator(device=dev).manual_seed(1)
    n = torch.randint(100, 1000, (K,), generator=g, device=dev).tolist()
    rows = torch.arange(K, dtype=torch.int32, device=dev)
    w = torch.tensor(n, dtype=torch.float32, device=dev)
    out = torch.empty(P, device=dev)
    tot = float(sum(n))
    res = {}
    for rep in range(1):
        for pad in (0, 3 * P + 256 * 7, 3 * P):
            ld = P + pad
            buf = torch.empty((K, ld), device=dev)
            buf.normal_(generator=g).mul_(0.05)
            f = lambda: _native.fedavg(buf, rows, w, tot, P, out)  # noqa: E731
            for _ in range(10):
                f()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(20):
                f()
            b.record()
            torch.cuda.synchronize()
            us = a.elapsed_time(b) / 20 * 1e3
            res.setdefault(pad, []).append(round(us, 1))
            del buf, f
            torch.cuda.empty_cache()
    for pad, v in res.items():
        gbs = [round((K * P * 4 + P * 4) / (u * 1e-6) / 1e9) for u in v]
        print(f"row pitch P+{pad}: {v} us  {gbs} GB/s", flush=True)


if __name__ == "__main__":
    main()
