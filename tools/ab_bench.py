#!/usr/bin/env python3
"""Same-process, interleaved A/B timing of libdls_hip.so variants (tools/_variants/).

    python tools/ab_bench.py --workloads fedavg,vote,quant,gemm,pack [--rounds 5]

Each variant library is loaded with its own ctypes handle; every round times
`--launches` launches of each variant back to back with HIP events, so box /
clock drift hits all variants alike (cdna_hip_programming.md §5.4 rule 24).
"""
import argparse
import ctypes
import glob
import json
import os
import statistics
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from distributed_learning_simulator_amd import _native  # noqa: E402
from distributed_learning_simulator_amd.layout import ParameterLayout  # noqa: E402
from distributed_learning_simulator_amd.model_shapes import resnet18_cifar, vgg16  # noqa: E402

P_ = ctypes.c_void_p


def load(path):
    L = ctypes.CDLL(path)
    # libraries named libdls_oldabi*.so predate nfast[4] (they take the fast-tile total)
    L.old_nfast = os.path.basename(path).startswith("libdls_oldabi")
    for name, (args, res) in _native.SIGNATURES.items():
        f = getattr(L, name, None)  # a variant built from an older tree may lack newer entry points
        if f is None:
            continue
        f.argtypes = args
        f.restype = res
    if L.old_nfast:
        L.dls_dequant_fedavg.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32] + \
            L.dls_dequant_fedavg.argtypes[3:]
    return L


def nfast_arg(L, counts):
    return int(sum(counts)) if L.old_nfast else (ctypes.c_int32 * len(counts))(*counts)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def setup(dev, want=()):
    W = {}
    lay = ParameterLayout(resnet18_cifar())
    P = lay.P
    g = torch.Generator(device=dev).manual_seed(1)
    U = torch.randn((100, P), generator=g, device=dev) * 0.05
    rows = torch.arange(100, dtype=torch.int32, device=dev)
    w = torch.randint(100, 1000, (100,), generator=g, device=dev).float()
    out = torch.empty(P, device=dev)
    tot = float(w.sum())
    W["fedavg"] = (lambda L: L.dls_fedavg_f32(ptr(U), P, ptr(rows), ptr(w), 100, tot, P, 0,
                                              ptr(out), stream()), 100 * P * 4 + P * 4)
    if "fedavg1k" in want:  # 1000 clients (45 GB of rows)
        U1 = torch.empty((1000, P), device=dev).normal_(generator=g).mul_(0.05)
        r1 = torch.arange(1000, dtype=torch.int32, device=dev)
        w1 = torch.randint(100, 1000, (1000,), generator=g, device=dev).float()
        t1 = float(w1.sum())
        W["fedavg1k"] = (lambda L: L.dls_fedavg_f32(ptr(U1), P, ptr(r1), ptr(w1), 1000, t1, P, 0,
                                                    ptr(out), stream()), 1000 * P * 4 + P * 4)
    if {"vote", "vote_sign", "pack"} & set(want):
        Wd = _native.sign_words(P)
        planes = torch.randint(-2**62, 2**62, (1000, _native.sign_row_pitch(P)), generator=g, device=dev)
        planes[:, 1::2] &= ~planes[:, 0::2]
        so = torch.empty(P, device=dev)
        cnt = torch.empty(P, dtype=torch.int32, device=dev)
        W["vote"] = (lambda L: L.dls_sign_vote(ptr(planes), planes.stride(0), None, 1000, P, ptr(cnt), ptr(so),
                                               None, stream()), 1000 * Wd * 8 + 2 * P * 4)
        vp = torch.empty(Wd, dtype=torch.int64, device=dev)
        W["vote_sign"] = (lambda L: L.dls_sign_vote(ptr(planes), planes.stride(0), None, 1000, P, None, ptr(so),
                                                    ptr(vp), stream()), 1000 * Wd * 8 + P * 4 + Wd * 8,
                          so)
        X = torch.sign(torch.randn((16, P), generator=g, device=dev))
        pk = torch.empty((16, Wd), dtype=torch.int64, device=dev)
        W["pack"] = (lambda L: L.dls_sign_pack_f32(ptr(X), P, 16, P, ptr(pk), Wd, None, stream()),
                     16 * (P * 4 + Wd * 8))
    if {"quant", "quant_fma", "quant1k", "quant_samerow", "quant_w0", "quant_w8",
            "quant_w16"} & set(want) or any(x.startswith("quant_fma") for x in want):
        from distributed_learning_simulator_amd.quant_store import QuantizedClientStore
        template = {}
        for name, s in vgg16():
            if len(s) >= 2:
                template[name] = (torch.zeros(s, dtype=torch.int8), torch.ones(s[0], dtype=torch.float64),
                                  torch.zeros(s[0], dtype=torch.int64))
            else:
                template[name] = torch.zeros(s)
        st = QuantizedClientStore(template, dev, capacity=100)
        st.Q.random_(0, 256, generator=g)
        st.F.normal_(generator=g)
        st.sz[..., 0].uniform_(1e-4, 1e-2, generator=g)
        st.sz[..., 1].zero_()
        qo = torch.empty(st.layout.P, device=dev)
        ql = st.qlayout
        Pq = sum(m for m, k in zip(st.layout.numels, ql.kinds) if k)
        Pf = sum(m for m, k in zip(st.layout.numels, ql.kinds) if not k)
        W["quant"] = (lambda L: L.dls_dequant_fedavg(ptr(st.tiles), st.ntiles, nfast_arg(L, st.nfast), ptr(st.Q), st.Q.stride(0),
                                                     ptr(st.F), st.F.stride(0), ptr(st.sz),
                                                     st.sz.stride(1) // 2, st.sz.stride(0) // 2,
                                                     ptr(rows), ptr(w), 100, tot,
                                                     ptr(qo), stream()),
                      100 * (Pq + 4 * Pf + 8 * ql.C) + 4 * st.layout.numel)
        # the same payloads with 1 KiB tiles only (FAST_TILE = TILE): the single-slice
        # kernel path, and the only tiling a library from before multi-KiB tiles handles
        from distributed_learning_simulator_amd import quant_store as qs
        saved, qs.FAST_TILE = qs.FAST_TILE, qs.TILE
        qt1, nf1 = ql.tiles()
        qs.FAST_TILE = saved
        tiles1 = torch.from_numpy(qt1.view(np.uint8).copy()).to(dev)
        W["quant1k"] = (lambda L: L.dls_dequant_fedavg(ptr(tiles1), len(qt1), nfast_arg(L, nf1), ptr(st.Q),
                                                       st.Q.stride(0), ptr(st.F), st.F.stride(0),
                                                       ptr(st.sz), st.sz.stride(1) // 2,
                                                       st.sz.stride(0) // 2, ptr(rows), ptr(w), 100,
                                                       tot, ptr(qo), stream()),
                        100 * (Pq + 4 * Pf + 8 * ql.C) + 4 * st.layout.numel)
        tf, ntf, nff = st.table(1)  # the FMA mode's tiling (quant_store.LANE_TILE_FMA)
        W["quant_fma"] = (lambda L: L.dls_dequant_fedavg_mode(
            ptr(tf), ntf, nfast_arg(L, nff), ptr(st.Q), st.Q.stride(0), ptr(st.F), st.F.stride(0),
            ptr(st.sz), st.sz.stride(1) // 2, st.sz.stride(0) // 2, ptr(rows), ptr(w), 100, tot, 1,
            ptr(qo), stream()), 100 * (Pq + 4 * Pf + 8 * ql.C) + 4 * st.layout.numel)
        # FMA tables with narrower tiles: one-channel FAST_TILE and the adaptive
        # lane widths capped at 2 / 1 KiB (for kernel builds with DLS_FMA_GMAX < 4)
        from distributed_learning_simulator_amd import quant_store as qsv

        def capped_table(qlay, cap):
            keep = (qsv.FAST_TILE, qsv.LANE_TILE_MAX)
            qsv.FAST_TILE, qsv.LANE_TILE_MAX = cap, cap
            tt, nft = qlay.tiles(qsv.LANE_TILE_FMA)
            qsv.FAST_TILE, qsv.LANE_TILE_MAX = keep
            return torch.from_numpy(tt.view(np.uint8).copy()).to(dev), len(tt), nft
        for cap in (3072, 2048, 1024):
            tc, ntc, nfc = capped_table(ql, cap)
            W[f"quant_fma_t{cap // 1024}"] = (
                lambda L, tc=tc, ntc=ntc, nfc=nfc: L.dls_dequant_fedavg_mode(
                    ptr(tc), ntc, nfast_arg(L, nfc), ptr(st.Q), st.Q.stride(0), ptr(st.F),
                    st.F.stride(0), ptr(st.sz), st.sz.stride(1) // 2, st.sz.stride(0) // 2,
                    ptr(rows), ptr(w), 100, tot, 1, ptr(qo), stream()),
                100 * (Pq + 4 * Pf + 8 * ql.C) + 4 * st.layout.numel, qo)
        if any(x.startswith("quant_fma_k300") for x in want):
            # 300 VGG-16 clients (41 GB): launch pieces 3x as long as at K = 100, the
            # per-piece fixed costs a third of the share
            st3 = QuantizedClientStore(template, dev, capacity=300)
            st3.Q.random_(0, 256, generator=g)
            st3.F.normal_(generator=g)
            st3.sz[..., 0].uniform_(1e-4, 1e-2, generator=g)
            st3.sz[..., 1].zero_()
            r3 = torch.arange(300, dtype=torch.int32, device=dev)
            w3 = torch.randint(100, 1000, (300,), generator=g, device=dev).float()
            t3 = float(w3.sum())
            for cap in (None, 2048, 1024):
                if cap is None:
                    tc, ntc, nfc = st3.table(1)
                    tag = ""
                else:
                    tc, ntc, nfc = capped_table(st3.qlayout, cap)
                    tag = f"_t{cap // 1024}"
                W["quant_fma_k300" + tag] = (
                    lambda L, tc=tc, ntc=ntc, nfc=nfc: L.dls_dequant_fedavg_mode(
                        ptr(tc), ntc, nfast_arg(L, nfc), ptr(st3.Q), st3.Q.stride(0), ptr(st3.F),
                        st3.F.stride(0), ptr(st3.sz), st3.sz.stride(1) // 2,
                        st3.sz.stride(0) // 2, ptr(r3), ptr(w3), 300, t3, 1, ptr(qo), stream()),
                    300 * (Pq + 4 * Pf + 8 * ql.C) + 4 * st.layout.numel, qo)
        # the FMA table's one-channel 4 KiB group alone (group 0: the fc layers) and
        # its lane groups alone: where the call's time goes
        tfh = ql.tiles(qsv.LANE_TILE_FMA, one_channel=True)
        toc, noc = ql.tiles(qsv.LANE_TILE_FMA, one_channel=True)  # the round-4 FMA table
        tocd = torch.from_numpy(toc.view(np.uint8).copy()).to(dev)
        W["quant_fma_oc"] = (lambda L: L.dls_dequant_fedavg_mode(
            ptr(tocd), len(toc), nfast_arg(L, noc), ptr(st.Q), st.Q.stride(0), ptr(st.F),
            st.F.stride(0), ptr(st.sz), st.sz.stride(1) // 2, st.sz.stride(0) // 2, ptr(rows),
            ptr(w), 100, tot, 1, ptr(qo), stream()),
            100 * (Pq + 4 * Pf + 8 * ql.C) + 4 * st.layout.numel, qo)
        tnew = ql.tiles(qsv.LANE_TILE_FMA, one_channel=False)
        keep8 = qsv.LANE_TILE_MAX
        qsv.LANE_TILE_MAX = 8192
        t8, n8 = ql.tiles(qsv.LANE_TILE_FMA, one_channel=False)
        qsv.LANE_TILE_MAX = keep8
        t8d = torch.from_numpy(t8.view(np.uint8).copy()).to(dev)
        W["quant_fma_w8"] = (lambda L: L.dls_dequant_fedavg_mode(
            ptr(t8d), len(t8), nfast_arg(L, n8), ptr(st.Q), st.Q.stride(0), ptr(st.F),
            st.F.stride(0), ptr(st.sz), st.sz.stride(1) // 2, st.sz.stride(0) // 2, ptr(rows),
            ptr(w), 100, tot, 1, ptr(qo), stream()),
            100 * (Pq + 4 * Pf + 8 * ql.C) + 4 * st.layout.numel, qo)
        for tag, lo, hi, tsrc in (("g0", 0, 1, tfh), ("lanes", 4, 8, tfh),
                                  ("int", 0, 8, tnew)):
            tt_, nf_ = tsrc
            a0, a1 = sum(nf_[:lo]), sum(nf_[:hi])
            sub = tt_[a0:a1]
            nsub = tuple(nf_[g] if lo <= g < hi else 0 for g in range(len(nf_)))
            td = torch.from_numpy(sub.view(np.uint8).copy()).to(dev)
            nbs = 100 * int(sub["len"].sum()) + 4 * int(((sub["len"] + 63) // 64 * 64).sum())
            W[f"quant_fma_{tag}"] = (
                lambda L, td=td, sub=sub, nsub=nsub: L.dls_dequant_fedavg_mode(
                    ptr(td), len(sub), nfast_arg(L, nsub), ptr(st.Q), st.Q.stride(0), ptr(st.F),
                    st.F.stride(0), ptr(st.sz), st.sz.stride(1) // 2, st.sz.stride(0) // 2,
                    ptr(rows), ptr(w), 100, tot, 1, ptr(qo), stream()), nbs, qo)
        rows0 = torch.zeros(100, dtype=torch.int32, device=dev)
        from distributed_learning_simulator_amd import quant_store as qs0
        for fwv in (0, 8, 16):
            fw0, qs0.FAST_WASTE = qs0.FAST_WASTE, fwv
            tvw, nfvw = st.qlayout.tiles()
            qs0.FAST_WASTE = fw0
            tvwd = torch.from_numpy(tvw.view(np.uint8).copy()).to(dev)
            W[f"quant_w{fwv}"] = (
                lambda L, tvwd=tvwd, tvw=tvw, nfvw=nfvw: L.dls_dequant_fedavg(
                    ptr(tvwd), len(tvw), nfast_arg(L, nfvw), ptr(st.Q), st.Q.stride(0), ptr(st.F),
                    st.F.stride(0), ptr(st.sz), st.sz.stride(1) // 2, st.sz.stride(0) // 2,
                    ptr(rows), ptr(w), 100, tot, ptr(qo), stream()),
                100 * (Pq + 4 * Pf + 8 * ql.C) + 4 * st.layout.numel)
        W["quant_samerow"] = (lambda L: L.dls_dequant_fedavg(ptr(st.tiles), st.ntiles, nfast_arg(L, st.nfast),
                                                             ptr(st.Q), st.Q.stride(0),
                                                             ptr(st.F), st.F.stride(0), ptr(st.sz),
                                                             st.sz.stride(1) // 2,
                                                             st.sz.stride(0) // 2, ptr(rows0), ptr(w),
                                                             100, tot, ptr(qo), stream()),
                              100 * (Pq + 4 * Pf + 8 * ql.C) + 4 * st.layout.numel)
    if any(w.startswith("quant_r18") for w in want):
        # north-star: 1000 ResNet-18 int8 updates; quant_r18_l1_w<N>: FAST_WASTE = N
        from distributed_learning_simulator_amd import quant_store as qs
        from distributed_learning_simulator_amd.quant_store import QuantizedClientStore as QCS
        template = {}
        for name, s in resnet18_cifar():
            if len(s) >= 2:
                template[name] = (torch.zeros(s, dtype=torch.int8), torch.ones(s[0], dtype=torch.float64),
                                  torch.zeros(s[0], dtype=torch.int64))
            else:
                template[name] = torch.zeros(s)
        sr = QCS(template, dev, capacity=1000)
        sr.Q.random_(0, 256, generator=g)
        sr.F.normal_(generator=g)
        sr.sz[..., 0].uniform_(1e-4, 1e-2, generator=g)
        sr.sz[..., 1].zero_()
        r1k = torch.arange(1000, dtype=torch.int32, device=dev)
        w1k = torch.randint(100, 1000, (1000,), generator=g, device=dev).float()
        t1k = float(w1k.sum())
        qo18 = torch.empty(sr.layout.P, device=dev)
        qlr = sr.qlayout
        nb = 1000 * (sum(m for m, k in zip(sr.layout.numels, qlr.kinds) if k) +
                     4 * sum(m for m, k in zip(sr.layout.numels, qlr.kinds) if not k) + 8 * qlr.C) \
            + 4 * sr.layout.numel
        saved = qs.LANE_TILE

        def table(lane_tile, f32_tile=None, small_tile=None, one_channel=True):
            keep = (qs.F32_TILE, qs.SMALL_TILE)
            qs.LANE_TILE = lane_tile
            qs.F32_TILE = f32_tile or keep[0]
            qs.SMALL_TILE = small_tile or keep[1]
            tt, nft = qlr.tiles(one_channel=one_channel)
            qs.LANE_TILE = saved
            qs.F32_TILE, qs.SMALL_TILE = keep
            return torch.from_numpy(tt.view(np.uint8).copy()).to(dev), tt, nft

        def qmode(tab, rows_t, w_t, tot, mode):
            tdev, tt, nft = tab
            return lambda L: L.dls_dequant_fedavg_mode(
                ptr(tdev), len(tt), nfast_arg(L, nft), ptr(sr.Q), sr.Q.stride(0), ptr(sr.F),
                sr.F.stride(0), ptr(sr.sz), sr.sz.stride(1) // 2, sr.sz.stride(0) // 2,
                ptr(rows_t), ptr(w_t), rows_t.numel(), tot, mode, ptr(qo18), stream())
        # the store's tilings (exact: LANE_TILE, FMA: LANE_TILE_FMA), 1 KiB and adaptive
        tab_p, tab_f = table(saved), table(qs.LANE_TILE_FMA, one_channel=qs.FMA_ONE_CHANNEL)
        # the FMA table's int groups alone (no fp32 / small-int side groups)
        tdf_, ttf_, nff_ = tab_f  # (names unique in setup(): the lambdas bind late)
        nint = sum(nff_[:8])
        tab_i = (tdf_, ttf_[:nint], tuple(nff_[:8]) + (0,) * (len(nff_) - 8))
        W["quant_r18_fma_int"] = (qmode(tab_i, r1k, w1k, t1k, 1), nb, qo18)
        tab_1, tab_a = table(1024), table("adaptive")
        W["quant_r18"] = (qmode(tab_p, r1k, w1k, t1k, 0), nb, qo18)
        W["quant_r18_l1"] = (qmode(tab_1, r1k, w1k, t1k, 0), nb, qo18)
        W["quant_r18_a"] = (qmode(tab_a, r1k, w1k, t1k, 0), nb, qo18)
        # DLS_FEDAVG_FMA (1e-6 tolerance mode) on the same 1000 clients
        W["quant_r18_fma"] = (qmode(tab_f, r1k, w1k, t1k, 1), nb, qo18)
        keep = qs.LANE_TILE_MAX
        qs.LANE_TILE_MAX = 8192
        W["quant_r18_fma_w8"] = (qmode(table(qs.LANE_TILE_FMA), r1k, w1k, t1k, 1), nb, qo18)
        qs.LANE_TILE_MAX = keep
        for cap in (3072, 2048, 1024):
            keep = (qs.FAST_TILE, qs.LANE_TILE_MAX)
            qs.FAST_TILE, qs.LANE_TILE_MAX = cap, cap
            tab_c = table(qs.LANE_TILE_FMA)
            qs.FAST_TILE, qs.LANE_TILE_MAX = keep
            W[f"quant_r18_fma_t{cap // 1024}"] = (qmode(tab_c, r1k, w1k, t1k, 1), nb, qo18)
        # the previous adaptive rule (4 / 2 / 1 KiB by row length, rows < 336 to the
        # small-int tiles): the tile-width policy A/B on the same kernels
        keep_rule = qs._adaptive_lane_tile
        qs._adaptive_lane_tile = lambda rl, n: (
            4096 if rl >= 2048 else 2048 if rl >= 1024 else 1024 if rl >= 336 else None)
        tab_old = table(qs.LANE_TILE_FMA)
        qs._adaptive_lane_tile = keep_rule
        W["quant_r18_fma_oldtab"] = (qmode(tab_old, r1k, w1k, t1k, 1), nb, qo18)
        # smaller fp32 / small-int tiles: more side-stream waves (latency-bound groups)
        for ft, stl in ((64, None), (64, 64), (128, 128)):
            tag = f"_f{ft}" + (f"s{stl}" if stl else "")
            W["quant_r18_fma" + tag] = (
                qmode(table(qs.LANE_TILE_FMA, ft, stl), r1k, w1k, t1k, 1), nb, qo18)
            W["quant_r18" + tag] = (qmode(table(saved, ft, stl), r1k, w1k, t1k, 0), nb, qo18)
        W["quant_r18_l1_fma"] = (qmode(tab_1, r1k, w1k, t1k, 1), nb, qo18)
        W["quant_r18_a_fma"] = (qmode(tab_a, r1k, w1k, t1k, 1), nb, qo18)
        # >= 10 ms dispatches for clock / counter probes: the 1000 client rows walked
        # 5 times (K = 5000, every pass from HBM: 11 GB >> L2 + MALL), and the same
        # arithmetic with every client on row 0 (payload loads L2-resident)
        r5k = r1k.repeat(5)
        w5k = w1k.repeat(5)
        t5k = float(w5k.sum())
        nb5 = 5 * (nb - 4 * sr.layout.numel) + 4 * sr.layout.numel
        W["quant_r18_k5000"] = (qmode(tab_p, r5k, w5k, t5k, 0), nb5)
        W["quant_r18_k5000_fma"] = (qmode(tab_f, r5k, w5k, t5k, 1), nb5)
        W["quant_r18_k5000_l2"] = (qmode(tab_p, torch.zeros_like(r5k), w5k, t5k, 0), nb5)
        # >= 10 ms lane-kernel dispatches (the clock quotient is validated there,
        # MI355X_MICROARCH.md DVFS): the rows walked 15 times
        r15k, w15k = r1k.repeat(15), w1k.repeat(15)
        t15k = float(w15k.sum())
        nb15 = 15 * (nb - 4 * sr.layout.numel) + 4 * sr.layout.numel
        W["quant_r18_k15000"] = (qmode(tab_p, r15k, w15k, t15k, 0), nb15)
        W["quant_r18_k15000_fma"] = (qmode(tab_p, r15k, w15k, t15k, 1), nb15)
        W["quant_r18_k15000_l2"] = (qmode(tab_p, torch.zeros_like(r15k), w15k, t15k, 0), nb15)
        tt, nft = tab_p[1], tab_p[2]
        if any(w.startswith("quant_r18_slab") for w in want):
            # slab-major emulation: every Q tile gets its own slab of 1000 consecutive
            # T-byte client pieces (ldq = T, src = slab start), so a wave streams its
            # slab sequentially; T = 1 KiB (1 KiB lane tiles) or 4 KiB (4 KiB lane tiles)
            for T, tag, lt in ((1024, "", 1024), (4096, "4", "adaptive")):
                _, tt, nft = table(lt)
                ts = tt.copy()
                isq = np.nonzero(ts["kind"] != 0)[0]
                ts["src"][isq] = np.arange(len(isq), dtype=np.int64) * 1000 * T
                Qs = torch.empty(len(isq) * 1000 * T, dtype=torch.uint8, device=dev)
                Qs.random_(0, 256, generator=g)
                tsd = torch.from_numpy(ts.view(np.uint8).copy()).to(dev)
                for mode, mtag in ((0, ""), (1, "_fma")):
                    W[f"quant_r18_slab{tag}{mtag}"] = (
                        lambda L, tsd=tsd, ts=ts, nft=nft, Qs=Qs, T=T, mode=mode:
                        L.dls_dequant_fedavg_mode(
                            ptr(tsd), len(ts), nfast_arg(L, nft), ptr(Qs), T, ptr(sr.F),
                            sr.F.stride(0), ptr(sr.sz), sr.sz.stride(1) // 2, sr.sz.stride(0) // 2,
                            ptr(r1k), ptr(w1k), 1000, t1k, mode, ptr(qo18), stream()), nb, qo18)
    # Shapley default path: 50 coalitions (members with p = 1/2) over 50 clients,
    # each client row read once per batch (dls_subset_fedavg_union_f32)
    from distributed_learning_simulator_amd.aggregation import union_batch
    gc = torch.Generator().manual_seed(5)
    member = torch.rand((50, 50), generator=gc) < 0.5
    member[:, 0] = True
    subs = [[k for k in range(50) if member[s, k]] for s in range(50)]
    nrow = {k: int(w[k]) for k in range(50)}
    ur, uwt, um, ut = union_batch(subs, nrow, dev)
    uo = torch.empty((50, P), device=dev)
    pairs = int(member.sum())
    uth = (ctypes.c_float * len(ut))(*ut)
    W["union"] = (lambda L: L.dls_subset_fedavg_union_f32(ptr(U), P, ptr(ur), ptr(uwt), ptr(um), 50,
                                                          uth, 50, P, ptr(uo), P, stream()),
                  100 * P * 4, uo)
    off, fr, fw, ft = [0], [], [], []
    for sub in subs:
        fr += sub
        fw += [nrow[k] for k in sub]
        ft.append(float(sum(nrow[k] for k in sub)))
        off.append(len(fr))
    t_off = torch.tensor(off, dtype=torch.int32, device=dev)
    t_fr = torch.tensor(fr, dtype=torch.int32, device=dev)
    t_fw = torch.tensor(fw, dtype=torch.float32, device=dev)
    t_ft = torch.tensor(ft, dtype=torch.float32, device=dev)
    W["subset_exact"] = (lambda L: L.dls_subset_fedavg_f32(ptr(U), P, ptr(t_off), ptr(t_fr),
                                                           ptr(t_fw), ptr(t_ft), 50, P, ptr(uo), P,
                                                           stream()), 100 * P * 4)
    print("union member pairs", pairs, flush=True)
    if "bn_act" in want:  # utility inference: eval BN + residual + ReLU, largest ResNet-18 activation
        bx = torch.randn(1000, 64, 32, 32, device=dev).contiguous(memory_format=torch.channels_last)
        br = torch.randn_like(bx)
        by = torch.empty_like(bx)
        bc = torch.cat([torch.randn(64, device=dev), torch.rand(64, device=dev) + 0.5,
                        torch.rand(64, device=dev) + 0.5, torch.randn(64, device=dev)])
        W["bn_act"] = (lambda L: L.dls_bn_act_exact_nhwc_f32(ptr(bx), 1000 * 32 * 32, 64, ptr(bc),
                                                              ptr(br), 1, ptr(by), stream()),
                       bx.numel() * 12)
    C = torch.rand((50, 50), generator=g, device=dev)
    C = C / C.sum(1, keepdim=True)
    go = torch.empty((50, P), device=dev)
    W["gemm"] = (lambda L: L.dls_subset_gemm_f32(ptr(C), 50, 50, ptr(U), P, ptr(rows), P, ptr(go),
                                                 P, stream()), 100 * P * 4)
    return W


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="fedavg,vote,quant,gemm,pack")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--launches", type=int, default=10)
    ap.add_argument("--only-run", action="store_true", help="just launch (rocprofv3 target)")
    ap.add_argument("--variants", default="",
                    help="comma-separated variant names (default: every lib in the directory)")
    ap.add_argument("--check", action="store_true",
                    help="workloads that name their output: every variant's bits equal the first's")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    libs = {os.path.basename(p)[7:-3]: load(p)
            for p in sorted(glob.glob(os.path.join(
                os.environ.get("DLS_VARIANTS", os.path.join(ROOT, "tools", "_variants")),
                "libdls_*.so")))}
    if args.variants:
        keep = args.variants.split(",")
        libs = {k: libs[k] for k in keep}
    W = setup(dev, args.workloads.split(","))
    res = {}
    for wl in args.workloads.split(","):
        fn, nbytes = W[wl][:2]
        if args.check and len(W[wl]) > 2:
            ref = None
            for name, L in libs.items():
                W[wl][2].fill_(float("nan"))
                assert fn(L) == 0
                torch.cuda.synchronize()
                got = W[wl][2].clone()
                if ref is None:
                    ref = got
                else:
                    same = torch.equal(got.view(torch.int32), ref.view(torch.int32))
                    print(wl, "check", name, "bit-identical" if same else "DIFFERS", flush=True)
                    assert same, (wl, name)
        if args.only_run:  # a profiler target: the first variant only, launches back to back
            L = next(iter(libs.values()))
            for _ in range(args.launches):
                assert fn(L) == 0
            torch.cuda.synchronize()
            print(wl, "ran", args.launches, flush=True)
            continue
        # warm (and check status): a variant that refuses the workload (e.g. a build
        # whose kernels do not take this table's tile widths) is skipped for it
        run = {}
        for name, L in libs.items():
            rc = fn(L)
            if rc != 0:
                print(wl, "skip", name, rc, L.dls_last_error().decode(), flush=True)
                continue
            run[name] = L
        torch.cuda.synchronize()
        times = {v: [] for v in run}
        for _ in range(args.rounds):
            for name, L in run.items():
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(args.launches):
                    fn(L)
                b.record()
                b.synchronize()
                times[name].append(a.elapsed_time(b) / args.launches)
        for name in run:
            ms = statistics.median(times[name])
            res.setdefault(wl, {})[name] = {"ms": round(ms, 4), "GBps": round(nbytes / ms / 1e6, 1),
                                           "min_ms": round(min(times[name]), 4)}
        print(wl, json.dumps(res[wl]), flush=True)


if __name__ == "__main__":
    main()
