#!/usr/bin/env python3
"""Do two utility forwards on two HIP streams overlap usefully?  Times N
ResNet-18 forward_split calls (the library's convolutions, 10k CIFAR-shaped
images each, two different random models alternating) issued on one stream vs
alternately on S streams, and checks that every forward's logits are the same
bits either way.

    python tools/stream_eval_probe.py [--images 10000] [--evals 8] [--streams 2] [--rounds 3]
"""
import argparse
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from distributed_learning_simulator_amd.models import ResNet18  # noqa: E402


def model(seed, dev):
    torch.manual_seed(seed)
    m = ResNet18().to(dev).eval()
    with torch.no_grad():
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm2d):
                mod.running_mean.uniform_(-0.2, 0.2)
                mod.running_var.uniform_(0.5, 2.0)
    return m


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=10000)
    ap.add_argument("--evals", type=int, default=8)
    ap.add_argument("--streams", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    X = torch.randn(a.images, 3, 32, 32, device=dev, generator=torch.Generator(device=dev).manual_seed(1))
    models = [model(s, dev) for s in range(2)]
    pks = [m.pack_split() for m in models]
    streams = [torch.cuda.Stream(dev) for _ in range(a.streams)]
    torch.cuda.synchronize()

    def run(nstreams):
        outs = [None] * a.evals
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if nstreams == 1:
            for i in range(a.evals):
                outs[i] = models[i % 2].forward_split(X, pks[i % 2])
        else:
            cur = torch.cuda.current_stream(dev)
            for s in streams[:nstreams]:
                s.wait_stream(cur)
            for i in range(a.evals):
                s = streams[i % nstreams]
                with torch.cuda.stream(s):
                    outs[i] = models[i % 2].forward_split(X, pks[i % 2])
            for s in streams[:nstreams]:
                cur.wait_stream(s)
        torch.cuda.synchronize()
        return time.perf_counter() - t0, outs

    ref = run(1)[1]  # warm-up + reference bits
    res = {1: [], a.streams: []}
    same = True
    for _ in range(a.rounds):
        for ns in (1, a.streams):
            el, outs = run(ns)
            res[ns].append(el)
            same &= all(torch.equal(o.view(torch.int32), r.view(torch.int32)) for o, r in zip(outs, ref))
    for ns, els in res.items():
        med = statistics.median(els)
        print(f"streams={ns}: {a.evals} forwards of {a.images} images: median {med * 1e3:.1f} ms "
              f"= {med / a.evals * 1e3:.2f} ms per forward = {a.evals / med:.2f} evals/s "
              f"(all: {', '.join(f'{e * 1e3:.1f}' for e in els)})")
    print(f"logits bit-identical across stream counts and rounds: {same}")


if __name__ == "__main__":
    main()
