#!/usr/bin/env python3
"""Probe: HBM write bandwidth of plain fills (torch zero_/fill_) over a [50, P]
ResNet-18-sized output, the subset GEMM's write volume."""
import torch


def main():
    dev = torch.device("cuda", 0)
    P = 11174016
    out = torch.empty((50, P), device=dev)
    for name, fn in (("zero_", lambda: out.zero_()), ("fill_", lambda: out.fill_(1.5))):
        for _ in range(5):
            fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(20):
            fn()
        b.record()
        b.synchronize()
        ms = a.elapsed_time(b) / 20
        print(f"{name}: {ms:.3f} ms, {out.numel() * 4 / ms / 1e6:.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
