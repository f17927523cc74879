#!/usr/bin/env python3
"""Probe: evaluating S subset models on one test set — S sequential forwards vs one
torch.func.vmap over the stacked parameters (grouped convolutions), fp32 NHWC."""
import copy
import os
import sys
import time

import torch
from torch.func import functional_call, stack_module_state

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from distributed_learning_simulator_amd.models import ResNet18  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    X = torch.randn(10000, 3, 32, 32, device=dev).contiguous(memory_format=torch.channels_last)
    base = ResNet18().to(dev).eval().to(memory_format=torch.channels_last)
    bs = int(os.environ.get("PROBE_BS", "1000"))
    for S in (1, 2, 4, 8):
        models = [copy.deepcopy(base) for _ in range(S)]
        for m in models:
            with torch.no_grad():
                for p in m.parameters():
                    p.add_(torch.randn_like(p) * 1e-3)

        def seq():
            out = 0
            with torch.no_grad():
                for m in models:
                    for i in range(0, X.shape[0], bs):
                        out += int((m(X[i:i + bs]).argmax(1) == 0).sum())
            return out

        nchw = [copy.deepcopy(m).to(memory_format=torch.contiguous_format) for m in models]
        params, buffers = stack_module_state(nchw)
        skel = copy.deepcopy(nchw[0]).to("meta")

        def f(p, b, x):
            return functional_call(skel, (p, b), (x,))

        vf = torch.vmap(f, in_dims=(0, 0, None))
        Xc = X.contiguous()  # vmap's batch-norm rule needs NCHW-contiguous inputs

        def vm():
            out = 0
            with torch.no_grad():
                for i in range(0, X.shape[0], bs):
                    out += int((vf(params, buffers, Xc[i:i + bs]).argmax(-1) == 0).sum())
            return out

        for name, fn in (("sequential", seq), ("vmap", vm)):
            fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            print(f"S={S} {name:10s}: {el / S * 1e3:7.1f} ms per model-eval ({S / el:.2f} evals/s)",
                  flush=True)


if __name__ == "__main__":
    main()
