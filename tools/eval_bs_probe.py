#!/usr/bin/env python3
"""Probe: one utility evaluation (ResNet-18, 10,000 CIFAR-shaped images, fp32 NHWC,
the fused eval forward) vs inference batch size and MIOpen's algorithm search."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from distributed_learning_simulator_amd.models import ResNet18  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    X = torch.randn(10000, 3, 32, 32, device=dev).contiguous(memory_format=torch.channels_last)
    m = ResNet18().to(dev).eval().to(memory_format=torch.channels_last)
    for bench in (False, True):
        torch.backends.cudnn.benchmark = bench
        for bs in (1000, 2000, 2500, 5000, 10000):
            fold = m.fold_bn()

            def ev():
                with torch.no_grad():
                    return [m.forward_fused(X[i:i + bs], fold).argmax(1) for i in range(0, 10000, bs)]
            ev()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                ev()
            torch.cuda.synchronize()
            print(f"benchmark={bench} bs={bs}: {(time.perf_counter() - t0) / 3 * 1e3:.1f} ms per eval",
                  flush=True)


if __name__ == "__main__":
    main()
