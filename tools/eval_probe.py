#!/usr/bin/env python3
"""Probe: fp32 ResNet-18 (CIFAR) inference throughput on 10k images under
memory formats / batch sizes / MIOpen benchmark mode (Shapley utility evals)."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from distributed_learning_simulator_amd.models import ResNet18  # noqa: E402


def run(model, X, bs, reps=3, fused=False):
    fwd = model
    if fused:  # models.ResNet18.forward_fused: hand-written eval batch norm + ReLU (+ residual)
        fold = model.fold_bn()
        fwd = lambda x: model.forward_fused(x, fold)  # noqa: E731
    with torch.no_grad():
        for i in range(0, X.shape[0], bs):
            fwd(X[i:i + bs]).argmax(1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            for i in range(0, X.shape[0], bs):
                fwd(X[i:i + bs]).argmax(1)
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    X = torch.randn(10000, 3, 32, 32, device=dev)
    if "--fused" in sys.argv:  # channels_last + fused batch norm, by benchmark mode and batch
        for bench in (False, True):
            torch.backends.cudnn.benchmark = bench
            model = ResNet18().to(dev).eval().to(memory_format=torch.channels_last)
            Xm = X.contiguous(memory_format=torch.channels_last)
            for bs in (500, 1000, 2000, 2500):
                el = run(model, Xm, bs, fused=True)
                print(f"fused benchmark={bench} batch={bs}: {el * 1e3:.1f} ms/eval "
                      f"({1 / el:.2f} evals/s)", flush=True)
        return
    for bench in (False, True):
        torch.backends.cudnn.benchmark = bench
        for cl in (False, True):
            model = ResNet18().to(dev).eval()
            Xm = X
            if cl:
                model = model.to(memory_format=torch.channels_last)
                Xm = X.contiguous(memory_format=torch.channels_last)
            for bs in (1000, 2500, 5000, 10000):
                el = run(model, Xm, bs)
                print(f"benchmark={bench} channels_last={cl} batch={bs}: {el * 1e3:.1f} ms/eval "
                      f"({1 / el:.2f} evals/s)", flush=True)


if __name__ == "__main__":
    main()
