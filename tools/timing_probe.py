#!/usr/bin/env python3
"""Probe: FedAvg (K=100 ResNet-18) kernel time vs how the client rows are allocated.

Separate torch allocations of the same size vs slices of one large allocation,
each timed with one event pair around 20 back-to-back launches.
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from distributed_learning_simulator_amd import _native  # noqa: E402
from distributed_learning_simulator_amd.layout import ParameterLayout  # noqa: E402
from distributed_learning_simulator_amd.model_shapes import resnet18_cifar  # noqa: E402


def time_fedavg(buf, rows, w, tot, P, out):
    for _ in range(10):
        _native.fedavg(buf, rows, w, tot, P, out)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        _native.fedavg(buf, rows, w, tot, P, out)
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / 20 * 1e3


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
    order = os.environ.get("PROBE_ORDER", "sep,big").split(",")
    for what in order:
        if what == "sep":
            sep, keep = [], []
            for i in range(6):
                buf = torch.empty((K, P), device=dev)
                buf.normal_(generator=g).mul_(0.05)
                sep.append(round(time_fedavg(buf, rows, w, tot, P, out), 1))
                keep.append(buf)  # keep them alive: every allocation is new memory
            print("separate 4.5 GB allocations (us):", sep, flush=True)
            del keep
        else:
            big = torch.empty((8 * K, P), device=dev)
            big.normal_(generator=g).mul_(0.05)
            sl = [round(time_fedavg(big[i * K:(i + 1) * K], rows, w, tot, P, out), 1)
                  for i in range(8)]
            print("slices of one 36 GB allocation (us):", sl, flush=True)
            del big
        torch.cuda.empty_cache()

if __name__ == "__main__":
    main()
