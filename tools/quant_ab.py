#!/usr/bin/env python3
"""Interleaved timing of dls_dequant_fedavg on 1000 x ResNet-18 int8 (and 100 x
VGG-16) for store-layout knobs: LANE_TILE (lane-tile width) and, with
DLS_HIP_LIB-style variant libraries, kernel builds.

    python tools/quant_ab.py --lane 1024,2048,4096 [--reps 5] [--check]

--check compares every width's output bit for bit with the first's.
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from distributed_learning_simulator_amd import _native, quant_store  # noqa: E402
from distributed_learning_simulator_amd.model_shapes import resnet18_cifar, vgg16  # noqa: E402


def make_store(shapes, K, lane_tile, dev, seed=5):
    quant_store.LANE_TILE = lane_tile
    template = {}
    for name, s in shapes:
        if len(s) >= 2:
            template[name] = (torch.zeros(s, dtype=torch.int8), torch.ones(s[0], dtype=torch.float64),
                              torch.zeros(s[0], dtype=torch.int64))
        else:
            template[name] = torch.zeros(s)
    st = quant_store.QuantizedClientStore(template, dev, capacity=K)
    g = torch.Generator(device=dev).manual_seed(seed)
    st.Q.random_(0, 256, generator=g)
    st.F.normal_(generator=g).mul_(0.01)
    st.sz[..., 0].uniform_(1e-4, 1e-2, generator=g)
    st.sz[..., 1].zero_()
    return st


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lane", default="1024,2048,4096")
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--K", type=int, default=1000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--launches", type=int, default=10)
    ap.add_argument("--check", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    shapes = resnet18_cifar() if args.model == "resnet18" else vgg16()
    lanes = [int(x) for x in args.lane.split(",")]
    st = make_store(shapes, args.K, lanes[0], dev)
    tables = {}
    for lt in lanes:
        quant_store.LANE_TILE = lt
        t, nf = st.qlayout.tiles()
        import numpy as np
        tables[lt] = (torch.from_numpy(t.view(np.uint8).copy()).to(dev), len(t), nf)
    K = args.K
    n = torch.randint(100, 1001, (K,), generator=torch.Generator().manual_seed(1)).tolist()
    rows = torch.arange(K, dtype=torch.int32, device=dev)
    w = torch.tensor(n, dtype=torch.float32, device=dev)
    total = float(sum(n))
    cases = [(lt, 0) for lt in lanes]
    outs = {c: torch.empty(st.layout.P, device=dev) for c in cases}
    ql = st.qlayout
    Pq = sum(m for m, k in zip(st.layout.numels, ql.kinds) if k)
    Pf = sum(m for m, k in zip(st.layout.numels, ql.kinds) if not k)
    nbytes = K * (Pq + 4 * Pf + 8 * ql.C) + 4 * st.layout.numel
    res = {c: [] for c in cases}
    for r in range(args.reps):
        for c in cases:
            lt = c[0]
            tb, nt, nf = tables[lt]
            for _ in range(2):
                _native.dequant_fedavg(tb, nt, nf, st.Q, st.F, st.sz, rows, w, total, outs[c])
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(args.launches):
                _native.dequant_fedavg(tb, nt, nf, st.Q, st.F, st.sz, rows, w, total, outs[c])
            b.record()
            torch.cuda.synchronize()
            res[c].append(a.elapsed_time(b) / args.launches)
    for c in cases:
        ms = sorted(res[c])[len(res[c]) // 2]
        print(f"lane_tile {c[0]}: nfast {tables[c[0]][2]} median {ms:.4f} ms  "
              f"{nbytes / ms / 1e6:.1f} GB/s  frac {nbytes / ms / 1e6 / 8000:.4f}  all {['%.4f' % x for x in res[c]]}",
              flush=True)
    if args.check:
        ref = outs[cases[0]]
        for c in cases[1:]:
            same = torch.equal(ref.view(torch.int32), outs[c].view(torch.int32))
            print(f"case {c} bit-identical to {cases[0]}: {same}", flush=True)


if __name__ == "__main__":
    main()
