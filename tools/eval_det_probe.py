#!/usr/bin/env python3
"""Probe: ResNet-18 (CIFAR) inference on 10k images with MIOpen deterministic
convolutions (torch.backends.cudnn.deterministic = True) vs its default
algorithms, NHWC vs NCHW — one configuration per process (MIOpen caches its
solution choice per problem in-process), so run it once per configuration:

    python tools/eval_det_probe.py {nhwc|nchw} {det|nondet} [fused]
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from distributed_learning_simulator_amd.models import ResNet18  # noqa: E402


def main():
    fmt, det = sys.argv[1], sys.argv[2] == "det"
    fused = "fused" in sys.argv[3:]
    dev = torch.device("cuda", 0)
    torch.backends.cudnn.deterministic = det
    torch.backends.cudnn.benchmark = False
    torch.manual_seed(0)
    X = torch.randn(10000, 3, 32, 32, device=dev)
    model = ResNet18().to(dev).eval()
    if fmt == "nhwc":
        model = model.to(memory_format=torch.channels_last)
        X = X.contiguous(memory_format=torch.channels_last)
    fwd = model
    if fused:
        fold = model.fold_bn()
        fwd = lambda x: model.forward_fused(x, fold)  # noqa: E731
    with torch.no_grad():
        t0 = time.perf_counter()
        fwd(X[:1000]).argmax(1)
        torch.cuda.synchronize()
        first = time.perf_counter() - t0
        t0 = time.perf_counter()
        out = torch.cat([fwd(X[i:i + 1000]) for i in range(0, 10000, 1000)])
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        out2 = torch.cat([fwd(X[i:i + 1000]) for i in range(0, 10000, 1000)])
        torch.cuda.synchronize()
    same = torch.equal(out.view(torch.int32), out2.view(torch.int32))
    print(f"{fmt} {'det' if det else 'nondet'}{' fused' if fused else ''}: first batch "
          f"{first:.2f} s, 10k images {el * 1e3:.1f} ms, repeat bit-identical {same}", flush=True)


if __name__ == "__main__":
    main()
