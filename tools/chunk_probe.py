#!/usr/bin/env python3
"""Probe: FedAvg (K=100 ResNet-18) time when the parameter range is reduced in
chunks (distributed.chunk_bounds, as the sharded server / multi-GPU bench do),
launches back to back on one stream, without the all-reduce."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from distributed_learning_simulator_amd import _native  # noqa: E402
from distributed_learning_simulator_amd.distributed import chunk_bounds  # noqa: E402
from distributed_learning_simulator_amd.layout import ParameterLayout  # noqa: E402
from distributed_learning_simulator_amd.model_shapes import resnet18_cifar  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    P = ParameterLayout(resnet18_cifar()).P
    K = 100
    g = torch.Generator(device=dev).manual_seed(1)
    U = torch.empty((K, P), device=dev).normal_(generator=g).mul_(0.05)
    rows = torch.arange(K, dtype=torch.int32, device=dev)
    w = torch.randint(100, 1000, (K,), generator=g, device=dev).float()
    tot = float(w.sum())
    out = torch.empty(P, device=dev)
    for chunks in (1, 2, 3, 4, 6, 8):
        b = chunk_bounds(P, chunks)

        def run():
            for c in range(chunks):
                if b[c + 1] > b[c]:
                    _native.fedavg(U[:, b[c]:], rows, w, tot, b[c + 1] - b[c], out[b[c]:b[c + 1]])
        for _ in range(5):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            run()
        e1.record()
        e1.synchronize()
        print(f"chunks={chunks}: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us  bounds={b}", flush=True)


if __name__ == "__main__":
    main()
