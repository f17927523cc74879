#!/usr/bin/env python3
"""Benchmark of the server-side aggregation hot path on MI355X.

Headline (BASELINE.json ``metric``): client-update GB/s aggregated per FL round,
on BASELINE config 2 — FedAvg of 100 synthetic ResNet-18 (11,173,962 fp32)
client updates per GPU, bit-exact reference-order kernel.  One "step" = one
aggregation of the resident client rows (plus, for N > 1 GPUs, the RCCL
all-reduce of the partial sums; clients are sharded, K per rank: weak scaling).

The same JSON line carries:
  * ``roofline``     dominant kernel (dls_fedavg_f32): algorithmic bytes per
                     launch / its average duration from HIP events recorded on
                     the launch stream around every launch of the timed region;
  * ``cpu_baseline`` the reference's own torch op sequence (oracle restatement,
                     servers/fed_server.py:52-65) on this host's cores, bounded
                     sample, rank 0 at N = 1 only;
  * ``components``   the other BASELINE configs (sign vote 1000 x ResNet-18,
                     fed_quant 100 x VGG-16, Shapley subset GEMM 50 x ResNet-18),
                     each with its own roofline (skip with --quick).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--quick]
"""
import argparse
import json
import math
import os
import platform
import subprocess
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from distributed_learning_simulator_amd import _native  # noqa: E402
from distributed_learning_simulator_amd.layout import ParameterLayout  # noqa: E402
from distributed_learning_simulator_amd.distributed import allreduce_chunked, chunk_bounds  # noqa: E402
from distributed_learning_simulator_amd.model_shapes import resnet18_cifar, vgg16  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA (~2.5 PF)
# f32 VALU issue roof: 256 CUs x 4 SIMDs x 32 lanes per clock x 2.4 GHz = 78.6 T
# lane-ops/s (a v_pk_* op = 2 lane-ops per lane; MI355X_MICROARCH.md: the f32
# VALU peak is 64 FLOP/clk/SIMD with FMAs counted twice)
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12
SEED = 20250127


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


# Single-GPU components warm up for at least this long before their timed
# launches: a kernel's time ramps over its first ~20-40 back-to-back launches
# (tools/launch_series.py: the sign vote 0.453 ms median over launches 0-19,
# 0.417-0.419 from launch 40 on), so a 5-launch warmup timed the ramp.  The
# headline keeps exactly the CLI's W warmup steps (the driver's contract), and so
# do the sharded components (their launches hold collectives: every rank must run
# the same count).
COMPONENT_WARM_S = 0.1


def timed_launches(fn, steps, warmup, sync_all=None, warm_s=0.0):
    """Run fn() warmup+steps times (plus further untimed launches until warm_s
    seconds of warmup have passed); HIP events around every timed launch on the
    current stream.  Returns (wall_s, [kernel_ms...])."""
    t0 = time.perf_counter()
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    while time.perf_counter() - t0 < warm_s:
        for _ in range(4):
            fn()
        torch.cuda.synchronize()
    if sync_all:
        sync_all()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    t0 = time.perf_counter()
    for a, b in ev:
        fn(a, b)
    torch.cuda.synchronize()
    if sync_all:
        sync_all()
    wall = time.perf_counter() - t0
    return wall, [a.elapsed_time(b) for a, b in ev]


def load_pmc(key):
    """This workload's entry of the committed rocprofv3 PMC passes
    (profiles/pmc_traffic.json, tools/pmc_traffic.py), or {}."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            return json.load(f).get(key, {})
    except (OSError, ValueError):
        return {}


def load_traffic(key):
    """HBM bytes per launch of this workload's kernel from the PMC passes, if present."""
    return load_pmc(key).get("hbm_bytes_per_launch")


def valu_issue(kernel, key):
    """The VALU issue roof from counters, for kernels whose VALU stream is fp32
    arithmetic: the fraction of the 1024 SIMDs' cycles their VALU was busy while
    this workload's kernels ran, 4 x SQ_INSTS_VALU / (1024 x GRBM_GUI_ACTIVE / 8)
    (profiles/pmc_traffic.json).  The 4 cycles per wave64 instruction are measured
    (tools/valu_issue_probe.hip, profiles/r04a_valu_issue.txt): v_fma_f32,
    v_pk_fma_f32, v_pk_mul_f32 and v_cvt_f32_ubyte issue at 4.0-4.3 SIMD cycles
    per wave-instruction with the SIMD saturated, but 32-bit integer / logic ops
    (v_xor_b32, v_add_u32, v_bitop3_b32) at ~2.5, so the formula overstates an
    integer-heavy kernel (the sign kernels read 1.1 in round 3) and is not
    reported for them.  None without the SQ pass."""
    f = load_pmc(key).get("valu_busy_frac")
    if f is None:
        return None
    return {"kernel": kernel, "bound": "valu_issue", "achieved": round(f, 4), "peak": 1.0,
            "unit": "VALU-busy fraction of SIMD cycles", "frac": round(f, 4),
            "source": "rocprofv3 SQ_ACTIVE_INST_VALU, GRBM_GUI_ACTIVE (profiles/pmc_traffic.json)"}


def roofline(kernel, bytes_per_launch, kernel_ms, bound="hbm", flops_per_launch=None, key=None):
    avg_s = sum(kernel_ms) / len(kernel_ms) / 1e3
    if bound == "hbm":
        achieved = bytes_per_launch / avg_s / 1e9
        peak, unit = HBM_PEAK_GBS, "GB/s"
    elif bound == "valu":  # flops_per_launch = f32 VALU lane-ops at the minimum op count
        achieved = flops_per_launch / avg_s / 1e12
        peak, unit = VALU_PEAK_TOPS, "T lane-op/s"
    else:
        achieved = flops_per_launch / avg_s / 1e12
        peak, unit = FP32_MFMA_PEAK_TFLOPS, "TFLOP/s"
    return {"kernel": kernel, "bound": bound, "achieved": round(achieved, 2), "peak": round(peak, 1),
            "unit": unit, "frac": round(achieved / peak, 4),
            "traffic": load_traffic(key) if key else None,
            "algorithmic_bytes_per_launch": bytes_per_launch,
            "avg_launch_us": round(avg_s * 1e6, 2)}


def synth_updates(K, P, dev, seed):
    """U_i = base + sigma_i * N(0,1), base ~ N(0, 0.05^2),
    sigma_i log-uniform in [1e-3, 5e-2], n_i ~ U{100..1000}."""
    g = torch.Generator(device=dev).manual_seed(seed)
    U = torch.empty((K, P), dtype=torch.float32, device=dev)
    U.normal_(generator=g)
    base = torch.randn(P, generator=g, device=dev) * 0.05
    lo, hi = math.log(1e-3), math.log(5e-2)
    sig = torch.exp(lo + (hi - lo) * torch.rand(K, generator=g, device=dev))
    U.mul_(sig[:, None]).add_(base[None, :])
    n = torch.randint(100, 1001, (K,), generator=g, device=dev).tolist()
    return U, n


# ----------------------------------------------------------------- FedAvg
def bench_fedavg(args, dev, rank, world, scaling="weak"):
    """Config 2.  weak: args.clients clients per GPU; strong: args.clients clients in
    total, dealt round-robin over the ranks (worker_id % world, simulator.py:68)."""
    layout = ParameterLayout(resnet18_cifar())
    P = layout.P
    K = args.clients if scaling == "weak" else len(range(rank, args.clients, world))
    U, n = synth_updates(K, P, dev, SEED + 1 + rank)
    # global sample count (FedAvg over all ranks' clients)
    n_all = torch.tensor([sum(n)], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(n_all)
    total = float(n_all.item())
    rows = torch.arange(K, dtype=torch.int32, device=dev)
    w = torch.tensor(n, dtype=torch.float32, device=dev)
    out = torch.empty(P, dtype=torch.float32, device=dev)
    chunks = args.chunks if world > 1 else 1
    bounds = chunk_bounds(P, chunks)  # decreasing sizes: the exposed last all-reduce is small
    kms = []

    def step(a=None, b=None):
        handles = []
        for c in range(chunks):
            c0, c1 = bounds[c], bounds[c + 1]
            if a is not None and c == 0:
                a.record()
            _native.fedavg(U[:, c0:], rows, w, total, c1 - c0, out[c0:c1])
            if b is not None and c == chunks - 1:
                b.record()
            if world > 1:
                handles.append(dist.all_reduce(out[c0:c1], async_op=True))
        for h in handles:
            h.wait()

    sync_all = dist.barrier if world > 1 else None
    wall, kms = timed_launches(step, args.steps, args.warmup, sync_all)
    t = torch.tensor([wall], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall = float(t.item())
    ms = wall / args.steps * 1e3
    upd_bytes = layout.numel * 4  # one client update (fp32, unpadded)
    total_clients = world * K if scaling == "weak" else args.clients
    value = total_clients * upd_bytes / (ms / 1e3) / 1e9
    bytes_per_launch = K * P * 4 + P * 4
    rf = roofline("dls_fedavg_f32", bytes_per_launch, kms,
                  key="headline" if scaling == "weak" and world == 1 else None)
    if world > 1:  # the events bracket all chunks' kernels (and interleaved RCCL enqueue)
        rf["note"] = "launch window includes chunked all-reduce overlap"
    del U
    return value, ms, rf, {"clients_per_gpu": K, "clients_total": total_clients,
                           "params": layout.numel, "padded_row": P}


def bench_fedavg_bitexact_sharded(args, dev, world, rank):
    """Config 2 strong scaling through ShardedFedServer(exchange="alltoall"): the
    bit-exact multi-GPU round (parameter slices per rank, one all-to-all of the
    client rows, the reference-order kernel over all clients per slice, one
    all-gather); args.clients clients in total, dealt worker_id % world."""
    from distributed_learning_simulator_amd.distributed import ShardedFedServer
    shapes = resnet18_cifar()
    server = ShardedFedServer(tester=None, worker_number=args.clients, synchronous=True,
                              device=dev, exchange="alltoall")
    g = torch.Generator(device=dev).manual_seed(SEED + 11 + rank)
    for wid in server.local_worker_ids:
        d = {k: torch.randn(sh, generator=g, device=dev) * 0.05 for k, sh in shapes}
        server.parameters[wid] = (100 + 9 * wid, d)
    ids = list(server.parameters.keys())

    def step(a=None, b=None):
        if a is not None:
            a.record()
        server.get_subset_model(ids)
        if b is not None:
            b.record()

    wall, _ = timed_launches(step, max(3, args.steps // 4), 2, dist.barrier)
    t = torch.tensor([wall], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ms = float(t.item()) / max(3, args.steps // 4) * 1e3
    numel = sum(math.prod(sh) for _, sh in shapes)
    del server
    return {"config": f"FedAvg of {args.clients} ResNet-18 updates in total over {world} GPUs, "
                      "bit-exact for any rank count (all-to-all of parameter slices + all-gather)",
            "value": round(args.clients * numel * 4 / (ms / 1e3) / 1e9, 2), "unit": "GB/s",
            "ms_per_step": round(ms, 4), "scaling": "strong"}


# ------------------------------------------------------------ components
def bench_fedavg_k1000(args, dev):
    """North-star scale: FedAvg of 1000 ResNet-18-sized updates (44.7 GB in HBM)."""
    layout = ParameterLayout(resnet18_cifar())
    P, K = layout.P, 1000
    U, n = synth_updates(K, P, dev, SEED + 7)
    rows = torch.arange(K, dtype=torch.int32, device=dev)
    w = torch.tensor(n, dtype=torch.float32, device=dev)
    out = torch.empty(P, device=dev)
    total = float(sum(n))

    def step(a=None, b=None):
        if a is not None:
            a.record()
        _native.fedavg(U, rows, w, total, P, out)
        if b is not None:
            b.record()

    wall, kms = timed_launches(step, max(3, args.steps // 4), 2, warm_s=COMPONENT_WARM_S)
    ms = wall / max(3, args.steps // 4) * 1e3
    del U
    return {"config": "FedAvg of 1000 ResNet-18 fp32 updates (44.7 GB), bit-exact reference order",
            "value": round(K * layout.numel * 4 / (ms / 1e3) / 1e9, 2), "unit": "GB/s",
            "ms_per_step": round(ms, 4),
            "roofline": roofline("dls_fedavg_f32", K * P * 4 + P * 4, kms, key="fedavg_k1000")}


def bench_sign(args, dev):
    layout = ParameterLayout(resnet18_cifar())
    P, K = layout.P, 1000
    W = _native.sign_words(P)
    g = torch.Generator(device=dev).manual_seed(SEED + 3)
    # the server's store layout: rows of W words at a 128-byte pitch
    planes = torch.randint(-2**62, 2**62, (K, _native.sign_row_pitch(P)), generator=g, device=dev)
    planes[:, 1::2] &= ~planes[:, 0::2]
    sign_out = torch.empty(P, device=dev)
    vote = torch.empty(W, dtype=torch.int64, device=dev)

    def step(a=None, b=None):  # the single-device server's launch (SignSGDServer)
        if a is not None:
            a.record()
        _native.sign_vote(planes, None, K, P, sign_out, vote_planes=vote)
        if b is not None:
            b.record()

    wall, kms = timed_launches(step, args.steps, args.warmup, warm_s=COMPONENT_WARM_S)
    ms = wall / args.steps * 1e3
    wire = W * 8
    bytes_per_launch = K * wire + P * 4 + wire  # client planes in, fp32 signs + packed vote out
    # worker/server pack kernel: fp32 signs -> planes, 16 clients per launch
    X = torch.sign(torch.randn((16, P), generator=g, device=dev))
    pk = torch.empty((16, W), dtype=torch.int64, device=dev)

    def pstep(a=None, b=None):
        if a is not None:
            a.record()
        _native.sign_pack(X, P, pk)
        if b is not None:
            b.record()

    _, pkms = timed_launches(pstep, args.steps, args.warmup, warm_s=COMPONENT_WARM_S)
    del planes, X
    return {
        "config": "signSGD majority vote, 1000 clients x ResNet-18 (2-bit planes in; fp32 "
                  "signs + packed vote out, one launch)",
        "value": round(K * wire / (ms / 1e3) / 1e9, 2), "unit": "GB/s (packed client updates)",
        "fp32_logical_GBps": round(K * layout.numel * 4 / (ms / 1e3) / 1e9, 2),
        "ms_per_step": round(ms, 4),
        "roofline": roofline("dls_sign_vote", bytes_per_launch, kms, key="sign_vote"),
        "pack": roofline("dls_sign_pack_f32", 16 * (P * 4 + W * 8), pkms, key="sign_pack"),
    }


def _quant_store(dev, K, seed, shapes=None):
    """K synthetic int8 payloads (per-channel symmetric weights, fp32 1-d tensors) of
    the given model (default VGG-16) in a device store."""
    from distributed_learning_simulator_amd.quant_store import QuantizedClientStore
    template = {}
    for name, s in (shapes or vgg16()):
        if len(s) >= 2:
            template[name] = (torch.zeros(s, dtype=torch.int8), torch.ones(s[0], dtype=torch.float64),
                              torch.zeros(s[0], dtype=torch.int64))
        else:
            template[name] = torch.zeros(s)
    store = QuantizedClientStore(template, dev, capacity=K)
    g = torch.Generator(device=dev).manual_seed(seed)
    store.Q.random_(0, 256, generator=g)  # int8 payload bytes
    store.F.normal_(generator=g).mul_(0.01)
    store.sz[..., 0].uniform_(1e-4, 1e-2, generator=g)
    store.sz[..., 1].zero_()
    store._free = []
    n = torch.randint(100, 1001, (K,), generator=g, device=dev).tolist()
    ql = store.qlayout
    Pq = sum(m for m, k in zip(store.layout.numels, ql.kinds) if k)
    Pf = sum(m for m, k in zip(store.layout.numels, ql.kinds) if not k)
    return store, n, Pq + 4 * Pf + 8 * ql.C, Pq + Pf


# ------------------------------------------------- sharded servers (N > 1)
def _max_over_ranks(wall, dev):
    t = torch.tensor([wall], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def bench_sign_sharded(args, dev, world, rank):
    """ShardedSignSGDServer's round (distributed.py): every rank votes its own 1000
    clients into int32 counts, RCCL int32 SUM all-reduce, counts -> fp32 signs +
    packed vote on every rank.  Weak scaling: 1000 clients per GPU."""
    layout = ParameterLayout(resnet18_cifar())
    P, K = layout.P, 1000
    W = _native.sign_words(P)
    g = torch.Generator(device=dev).manual_seed(SEED + 30 + rank)
    planes = torch.randint(-2**62, 2**62, (K, _native.sign_row_pitch(P)), generator=g, device=dev)
    planes[:, 1::2] &= ~planes[:, 0::2]
    counts = torch.empty(P, dtype=torch.int32, device=dev)
    sign_out = torch.empty(P, device=dev)
    vote = torch.empty(W, dtype=torch.int64, device=dev)

    def step(a=None, b=None):
        if a is not None:
            a.record()
        _native.sign_vote_count(planes, None, K, P, counts)
        if b is not None:
            b.record()
        dist.all_reduce(counts)
        _native.sign_from_counts(counts, P, sign_out, vote)

    wall, kms = timed_launches(step, args.steps, args.warmup, dist.barrier)
    ms = _max_over_ranks(wall, dev) / args.steps * 1e3
    del planes
    return {"config": f"signSGD majority vote sharded over {world} GPUs: 1000 clients x ResNet-18 "
                      "per GPU, int32 counts + RCCL all-reduce + signs / packed vote on every rank",
            "value": round(world * K * W * 8 / (ms / 1e3) / 1e9, 2),
            "unit": "GB/s (packed client updates, all ranks)", "ms_per_step": round(ms, 4),
            "count_kernel_us": round(sum(kms) / len(kms) * 1e3, 2)}


def bench_quant_sharded(args, dev, world, rank):
    """ShardedFedQuantServer's round: every rank dequant-averages its own 100 VGG-16
    clients with the global sample count, then a chunked fp32 SUM all-reduce of
    the 553 MB aggregate.  Weak scaling: 100 clients per GPU."""
    store, n, client_bytes, _ = _quant_store(dev, 100, SEED + 40 + rank)
    K = len(n)
    n_all = torch.tensor([sum(n)], dtype=torch.float64, device=dev)
    dist.all_reduce(n_all)
    total = float(n_all.item())
    out = torch.empty(store.layout.P, device=dev)
    rows_t = torch.arange(K, dtype=torch.int32, device=dev)
    w_t = torch.tensor(n, dtype=torch.float32, device=dev)

    def step(a=None, b=None):
        if a is not None:
            a.record()
        _native.dequant_fedavg(store.tiles, store.ntiles, store.nfast, store.Q, store.F, store.sz,
                               rows_t, w_t, total, out)
        if b is not None:
            b.record()
        allreduce_chunked(out, args.chunks)

    wall, kms = timed_launches(step, args.steps, args.warmup, dist.barrier)
    ms = _max_over_ranks(wall, dev) / args.steps * 1e3
    del store
    return {"config": f"fed_quant 8-bit sharded over {world} GPUs: 100 VGG-16 clients per GPU, "
                      "fused dequant + FedAvg, chunked RCCL fp32 all-reduce",
            "value": round(world * K * client_bytes / (ms / 1e3) / 1e9, 2),
            "unit": "GB/s (int8 client updates, all ranks)", "ms_per_step": round(ms, 4),
            "dequant_kernel_us": round(sum(kms) / len(kms) * 1e3, 2)}


def bench_quant(args, dev, K=100, shapes=None, model="VGG-16", key="fed_quant"):
    store, n, client_bytes, p_logical = _quant_store(dev, K, SEED + 4, shapes)
    out = torch.empty(store.layout.P, device=dev)
    rows_t = torch.arange(K, dtype=torch.int32, device=dev)
    w_t = torch.tensor(n, dtype=torch.float32, device=dev)
    total = float(sum(n))

    def stepper(mode):
        def step(a=None, b=None):
            if a is not None:
                a.record()
            tiles, ntiles, nfast = store.table(mode)
            _native.dequant_fedavg(tiles, ntiles, nfast, store.Q, store.F, store.sz, rows_t, w_t,
                                   total, out, mode=mode)
            if b is not None:
                b.record()
        return step

    steps = args.steps if K <= 100 else max(3, args.steps // 4)
    wall, kms = timed_launches(stepper(_native.FEDAVG_EXACT), steps, min(args.warmup, 3),
                               warm_s=COMPONENT_WARM_S)
    ms = wall / steps * 1e3
    bytes_per_launch = K * client_bytes + 4 * store.layout.numel
    # the FMA mode (DLS_FEDAVG_FMA: one constant per (client, channel), within the
    # north-star 1e-6 FedAvg tolerance, not bit-exact) on the same payloads
    fwall, fkms = timed_launches(stepper(_native.FEDAVG_FMA), steps, min(args.warmup, 3),
                                 warm_s=COMPONENT_WARM_S)
    fms = fwall / steps * 1e3
    # VALU roof at the reference's minimum op count: per int8 element and client
    # cvt + fl(q - zp)*s + *n_i + /N (two-constant: 2 ops, Markstein: 3) + add
    from distributed_learning_simulator_amd._native import two_constant_division
    div_ops = 2 if two_constant_division(total) else 3
    valu_ops = K * p_logical * (4 + div_ops)
    del store
    return {
        "config": f"fed_quant 8-bit, {K} clients x {model}, fused dequant + FedAvg (bit-exact)",
        "value": round(K * client_bytes / (ms / 1e3) / 1e9, 2),
        "unit": "GB/s (int8 client updates)",
        "fp32_logical_GBps": round(K * p_logical * 4 / (ms / 1e3) / 1e9, 2),
        "ms_per_step": round(ms, 4),
        "roofline": roofline("dls_dequant_fedavg", bytes_per_launch, kms, key=key),
        "valu_roof": roofline("dls_dequant_fedavg", bytes_per_launch, kms, bound="valu",
                              flops_per_launch=valu_ops),
        "valu_issue": valu_issue("dls_dequant_fedavg", key),
        "fma_mode": {
            "config": "the same payloads, dls_dequant_fedavg_mode DLS_FEDAVG_FMA: int8 tiles "
                      "accumulate fma(q, fl(fl(s*n_i)/N), acc) (normwise <= 1e-6 of the exact "
                      "aggregate, tests/test_gpu_quant.py)",
            "value": round(K * client_bytes / (fms / 1e3) / 1e9, 2),
            "unit": "GB/s (int8 client updates)", "ms_per_step": round(fms, 4),
            "roofline": roofline("dls_dequant_fedavg_mode", bytes_per_launch, fkms,
                                 key=key + "_fma"),
        },
    }


def bench_quant_k1000(args, dev):
    """North-star: quantized aggregation of 1000 ResNet-18-sized int8 updates."""
    return bench_quant(args, dev, K=1000, shapes=resnet18_cifar(), model="ResNet-18",
                       key="fed_quant_k1000")


CONFIG1 = dict(worker_number=10, rounds=5, train_size=60000, test_size=10000, epoch=1,
               batch_size=64, learning_rate=0.01)


def bench_config1(args, dev):
    """BASELINE config 1 end to end on the GPU: FedAvg, 10 workers (threads, as
    simulator.py:59-69), LeNet-5 on MNIST-shaped synthetic data (60,000 training /
    10,000 test images), 5 rounds, through simulator.run (the drop-in factory,
    queue, FedWorker, FedServer with the dls_fedavg_f32 aggregation and the
    tester).  Per-round wall time = time between consecutive aggregations (round 1
    from the start of the run, so it carries the workers' start-up)."""
    from distributed_learning_simulator_amd import simulator
    from distributed_learning_simulator_amd.servers.fed_server import FedServer
    c = CONFIG1
    cfg = simulator.get_config([
        "--distributed_algorithm", "fed", "--worker_number", str(c["worker_number"]),
        "--round", str(c["rounds"]), "--dataset_name", "MNIST", "--model_name", "LeNet5",
        "--epoch", str(c["epoch"]), "--batch_size", str(c["batch_size"]),
        "--learning_rate", str(c["learning_rate"]), "--train_size", str(c["train_size"]),
        "--test_size", str(c["test_size"]), "--log_dir", "", "--log_level", "WARNING"])
    stamps, agg_s = [], []
    orig = FedServer.get_subset_model

    def timed_subset(self, subset):
        t0 = time.perf_counter()
        out = orig(self, subset)
        torch.cuda.synchronize()
        agg_s.append(time.perf_counter() - t0)
        stamps.append(time.perf_counter())
        return out

    FedServer.get_subset_model = timed_subset
    try:
        t0 = time.perf_counter()
        # one process, this rank's GPU: inside a multi-rank job the default would pick
        # the sharded servers, whose collectives the other ranks never join
        server = simulator.run(cfg, devices=[dev], sharded=False)
        wall = time.perf_counter() - t0
    finally:
        FedServer.get_subset_model = orig
    rounds = [b - a for a, b in zip([t0] + stamps[:-1], stamps)]
    acc = server.get_metric(server.prev_model)
    return {"config": "FedAvg, 10 workers, LeNet-5 on MNIST-shaped synthetic data (60k train / "
                      "10k test), 5 rounds, simulator.run on 1 GPU (worker threads + server)",
            "value": round(sum(rounds[1:]) / max(1, len(rounds) - 1), 4),
            "unit": "s per round (rounds 2-5)", "higher_is_better": False,
            "round_s": [round(r, 4) for r in rounds], "wall_s": round(wall, 3),
            "aggregation_ms": [round(a * 1e3, 3) for a in agg_s],
            "rounds": server.round, "test_accuracy": acc}


def cpu_config1(args, threads):
    """BASELINE config 1 on the host cores: the reference's FedAvg simulator loop
    restated (oracle/simulator.py), same model, data shapes, split and
    hyper-parameters as bench_config1; bounded to about args.cpu_seconds."""
    from distributed_learning_simulator_amd.models import LeNet5, synthetic_classification
    from oracle.simulator import run_fedavg_cpu  # test infrastructure, timed only
    c = CONFIG1
    train = synthetic_classification(c["train_size"], (1, 32, 32), seed=0)
    test = synthetic_classification(c["test_size"], (1, 32, 32), seed=1)
    times, accs = run_fedavg_cpu(LeNet5, train, test, c["worker_number"], c["rounds"],
                                 epoch=c["epoch"], batch_size=c["batch_size"],
                                 learning_rate=c["learning_rate"], max_seconds=args.cpu_seconds)
    # the GPU leg's window: rounds 2.. (round 1 carries start-up) whenever at least
    # two rounds ran within the time bound
    window = times[1:] if len(times) >= 2 else times
    first = 2 if len(times) >= 2 else 1
    return {"value": round(sum(window) / len(window), 4),
            "unit": f"s per round (rounds {first}-{len(times)})",
            "higher_is_better": False, "cores": threads, "kind": "port",
            "sample": f"{len(times)} of {c['rounds']} rounds ran (10 workers x 6,000 images, "
                      f"LeNet-5); value over {len(window)} round(s)",
            "round_s": [round(t, 3) for t in times], "test_accuracy": accs[-1]}


def _shapley_coalitions(K, S, seed):
    """S coalitions of K clients, members with probability 1/2 (client 0 always),
    as sorted tuples (how the Shapley servers pass them)."""
    g = torch.Generator().manual_seed(seed)
    member = torch.rand((S, K), generator=g) < 0.5
    member[:, 0] = True
    return [tuple(k for k in range(K) if member[s, k]) for s in range(S)]


def bench_shapley_exact(args, dev):
    """Config 5a, the Shapley servers' default path: S bit-exact subset models of K
    clients in one dls_subset_fedavg_union_f32 launch (each client row read once)."""
    from distributed_learning_simulator_amd.aggregation import union_batch
    layout = ParameterLayout(resnet18_cifar())
    P, K, S = layout.P, 50, args.subsets
    U, n = synth_updates(K, P, dev, SEED + 5)
    subs = _shapley_coalitions(K, S, SEED + 5)
    t = union_batch([list(c) for c in subs], dict(enumerate(n)), dev)
    out = torch.empty((S, P), device=dev)

    def step(a=None, b=None):
        if a is not None:
            a.record()
        _native.subset_fedavg_union(U, *t, P, out)
        if b is not None:
            b.record()

    wall, kms = timed_launches(step, args.steps, args.warmup, warm_s=COMPONENT_WARM_S)
    ms = wall / args.steps * 1e3
    pairs = sum(len(c) for c in subs)
    # minimum VALU lane-ops: per parameter, per (client, coalition) membership the
    # quotient (two-constant 2 ops where proven for the coalition's N, else
    # Markstein's 3) + the add, and 1 per client for t = x * n_i
    from distributed_learning_simulator_amd._native import two_constant_division
    per_member = sum(len(c) * (1 + (2 if two_constant_division(float(sum(n[k] for k in c))) else 3))
                     for c in subs)
    valu_ops = layout.numel * (per_member + K)
    bytes_per_launch = (K + S) * P * 4
    # the per-coalition kernel on the same batch, for comparison
    off, fr, fw, ft = [0], [], [], []
    for c in subs:
        fr += c
        fw += [n[k] for k in c]
        ft.append(float(sum(n[k] for k in c)))
        off.append(len(fr))
    tt = [torch.tensor(v, dtype=dt, device=dev) for v, dt in
          ((off, torch.int32), (fr, torch.int32), (fw, torch.float32), (ft, torch.float32))]

    def step_pc(a=None, b=None):
        if a is not None:
            a.record()
        _native.subset_fedavg(U, *tt, P, out)
        if b is not None:
            b.record()

    _, kms_pc = timed_launches(step_pc, max(3, args.steps // 4), 1, warm_s=COMPONENT_WARM_S)
    del U, out
    return {
        "config": f"Shapley subset models, default bit-exact path: {S} coalitions (members p=1/2, "
                  f"{pairs} memberships) of 50 clients x ResNet-18, one union launch",
        "value": round(S / (ms / 1e3), 1), "unit": "subset models/s",
        "ms_per_step": round(ms, 4),
        "roofline": roofline("dls_subset_fedavg_union_f32", bytes_per_launch, kms,
                             key="shapley_exact"),
        "valu_roof": roofline("dls_subset_fedavg_union_f32", bytes_per_launch, kms, bound="valu",
                              flops_per_launch=valu_ops),
        "valu_issue": valu_issue("dls_subset_fedavg_union_f32", "shapley_exact"),
        "per_coalition_kernel_ms": round(sum(kms_pc) / len(kms_pc), 4),
    }


def bench_shapley_gemm(args, dev):
    layout = ParameterLayout(resnet18_cifar())
    P, K, S = layout.P, 50, args.subsets
    U, n = synth_updates(K, P, dev, SEED + 5)
    g = torch.Generator().manual_seed(SEED + 5)
    member = torch.rand((S, K), generator=g) < 0.5
    member[:, 0] = True
    nn_ = torch.tensor(n, dtype=torch.float64)
    C = (member.double() * nn_[None, :])
    C = (C / C.sum(1, keepdim=True)).float().to(dev)
    rows = torch.arange(K, dtype=torch.int32, device=dev)
    out = torch.empty((S, P), device=dev)

    def step(a=None, b=None):
        if a is not None:
            a.record()
        _native.subset_gemm(C, U, rows, P, out)
        if b is not None:
            b.record()

    wall, kms = timed_launches(step, args.steps, args.warmup, warm_s=COMPONENT_WARM_S)
    ms = wall / args.steps * 1e3
    flops = 2.0 * S * K * layout.numel
    bytes_per_launch = (K + S) * P * 4
    rf_hbm = roofline("dls_subset_gemm_f32", bytes_per_launch, kms, key="shapley_gemm")
    rf_mfma = roofline("dls_subset_gemm_f32", bytes_per_launch, kms, bound="mfma",
                       flops_per_launch=flops, key="shapley_gemm")
    del U, out
    return {
        "config": f"Shapley subset aggregation as fp32 MFMA GEMM, {S} subsets x 50 clients x ResNet-18",
        "value": round(S / (ms / 1e3), 1), "unit": "subset models/s",
        "ms_per_step": round(ms, 4), "roofline": rf_hbm, "mfma": rf_mfma,
    }


def _shapley_eval_server(args, dev, K=50):
    """A Shapley server (the servers' own evaluate_subsets path) with a ResNet-18
    tester on a CIFAR-10-shaped synthetic test set labelled by a fixed teacher, and
    K clients = teacher + client noise (so utilities differ)."""
    from distributed_learning_simulator_amd.model_util import ModelUtil
    from distributed_learning_simulator_amd.models import ResNet18
    from distributed_learning_simulator_amd.servers.shapley_value_server import ShapleyValueServer
    from distributed_learning_simulator_amd.trainer import Inferencer
    torch.manual_seed(SEED + 6)
    teacher = ResNet18().to(dev).eval()
    X = torch.randn(args.eval_images, 3, 32, 32, device=dev)
    with torch.no_grad():
        y = torch.cat([teacher(X[i:i + 1000]).argmax(1) for i in range(0, X.shape[0], 1000)])
    # the test set is handed over on the host, as simulator.py:68-74 builds the
    # tester (the Inferencer copies it to HBM once, on its first evaluation)
    X, y = X.cpu(), y.cpu()
    tester = Inferencer(ResNet18().to(dev), (X, y), batch_size=1000, device=dev)
    server = ShapleyValueServer(tester=tester, worker_number=K, synchronous=True, device=dev)
    base = ModelUtil(teacher).get_parameter_dict()
    g = torch.Generator(device=dev).manual_seed(SEED + 6)
    for wid in range(K):
        d = {k: v + torch.randn(v.shape, generator=g, device=dev) * 0.002 for k, v in base.items()}
        server.parameters[wid] = (100 + 17 * wid, d)
    return server


def conv_eval_roofline(tester, reps=3):
    """The utility forward's MFMA roof (csrc/conv.hip): forward_split over the
    tester's images (weights packed once, batches of tester.batch_size), timed with
    HIP events on the current stream (every launch of the forward runs there).
    achieved = issued bf16 MFMA flops (3 products x 2 x the MACs of the padded
    operands: the stem's 27 -> 32 im2col channels) / time, against the dense bf16
    peak; fp32_equivalent = the model's own 2 x MACs / time."""
    from distributed_learning_simulator_amd.models import split_conv_macs
    model, X = tester.model, tester.dataset[0]
    issued, useful = split_conv_macs(model, X.shape[2], X.shape[3])
    X = tester._resident_dataset()[0]
    n, bs = X.shape[0], tester.split_batch(X.shape[0])  # the Inferencer's own
    with torch.no_grad():
        pk = model.pack_split()
        for i in range(0, n, bs):
            model.forward_split(X[i:i + bs], pk)
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(0, n, bs):
                model.forward_split(X[i:i + bs], pk)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
    ms = sorted(ts)[len(ts) // 2]
    ach = 6 * issued * n / (ms / 1e3) / 1e12
    return {"kernel": "dls_conv_bn_act_split (k_conv3x3_pipe16, k_conv3x3s2_phase, k_conv_bf16x3, k_conv_stem) + pool_linear",
            "bound": "mfma", "achieved": round(ach, 1), "peak": BF16_MFMA_PEAK_TFLOPS,
            "unit": "TFLOP/s (bf16 MFMA issued)", "frac": round(ach / BF16_MFMA_PEAK_TFLOPS, 4),
            "traffic": None, "ms_per_forward_of_all_images": round(ms, 3),
            "issued_macs_per_image": issued, "model_macs_per_image": useful,
            "fp32_equivalent_tflops": round(2 * useful * n / (ms / 1e3) / 1e12, 1)}


def bench_shapley_evals(args, dev, world=1, rank=0):
    """Config 5b: Shapley utility evaluations through ShapleyValueServer.evaluate_subsets
    (batched bit-exact subset models + ResNet-18 test-set inference; on N ranks the
    coalitions are dealt round-robin and the utilities all-reduced).  Weak scaling:
    args.evals coalitions per GPU.  Timed with the tester's default GPU forward (the
    value: the library's deterministic convolutions, csrc/conv.hip — a coalition's
    utility is a function of the coalition in any process), and, for comparison,
    with MIOpen convolutions: its deterministic algorithms with the fused exact
    batch-norm pass (round 4's default, logits bit-identical to the module's
    forward), the module's own forward, and MIOpen's non-deterministic algorithms."""
    ts = time.perf_counter()
    server = _shapley_eval_server(args, dev)
    if rank == 0:
        log(f"shapley_evals: server and test set ready in {time.perf_counter() - ts:.1f} s")
    coal = _shapley_coalitions(50, (args.evals + 2) * world, SEED + 7)

    def timed(conv="dls", fused=True, deterministic=True):
        server.tester.conv = conv
        server.tester.fused_eval = fused
        server.tester.deterministic = deterministic
        tw = time.perf_counter()
        server.evaluate_subsets(coal[: 2 * world])  # kernel selection, warm caches
        torch.cuda.synchronize()
        if rank == 0:
            log(f"shapley_evals: warm-up (conv={conv}, fused={fused}, deterministic={deterministic}) "
                f"{time.perf_counter() - tw:.1f} s")
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        vals = server.evaluate_subsets(coal[2 * world:])
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        if rank == 0:
            log(f"shapley_evals: {len(coal) - 2 * world} evals in {el:.2f} s")
        if world > 1:
            el = _max_over_ranks(el, dev)
        return el, vals

    el, vals = timed()
    el_md, vals_md = timed("miopen")
    el_m, vals_m = timed("miopen", fused=False)
    # the cost of reproducible utilities on MIOpen: its default (not run-to-run
    # reproducible) algorithms
    el_nd, _ = timed("miopen", deterministic=False)
    server.tester.conv, server.tester.fused_eval, server.tester.deterministic = "dls", True, True
    n = len(coal) - 2 * world
    rf = conv_eval_roofline(server.tester) if rank == 0 else None
    split_batch = server.tester.split_batch(server.tester.dataset[0].shape[0])
    del server
    torch.cuda.empty_cache()
    bn = bench_bn_act(args, dev) if rank == 0 else None
    rate = lambda e: {"value": round(n / e, 3), "unit": "subset-evals/s (all GPUs)",  # noqa: E731
                      "ms_per_eval_per_gpu": round(e / n * world * 1e3, 2)}
    return {"config": f"Shapley utility evals via evaluate_subsets: {n} coalitions of 50 clients "
                      f"over {world} GPU(s), bit-exact subset models + ResNet-18 inference on "
                      f"{args.eval_images} CIFAR-10-shaped images handed to the tester on the host "
                      f"(copied to HBM once, on first use; tester batch 1000, forward "
                      f"batches of {split_batch}): the library's deterministic convolutions (bf16x3 MFMA, "
                      f"fused eval batch norm)",
            **rate(el),
            "utility_range": [round(min(vals), 4), round(max(vals), 4)],
            "deterministic_convs": True,
            "roofline": rf,
            "miopen_deterministic": {**rate(el_md), "max_utility_diff": round(
                max(abs(a - b) for a, b in zip(vals, vals_md)), 6),
                "note": "Inferencer(conv='miopen'): MIOpen's deterministic NCHW convolutions + "
                        "the fused exact batch-norm pass (round 4's default; logits "
                        "bit-identical to the module's forward)"},
            "module_forward": {**rate(el_m), "max_utility_diff_vs_miopen_deterministic": round(
                max(abs(a - b) for a, b in zip(vals_md, vals_m)), 6),
                "note": "Inferencer(conv='miopen', fused_eval=False): the module's own eval "
                        "forward (MIOpen convolutions and batch norm, separate add and ReLU)"},
            "nondeterministic_convs": {**rate(el_nd),
                                       "note": "MIOpen's default (not run-to-run reproducible) "
                                               "convolution algorithms on NHWC activations"},
            "bn_act": bn}


def bench_bn_act(args, dev):
    """The utility inference's hand-written pass (dls_bn_act_exact_nhwc_f32): eval
    batch norm + residual add + ReLU over ResNet-18's largest activation, a batch
    of 1000 CIFAR images x 64 channels x 32 x 32 (channels_last); 12 B per element."""
    x = torch.randn(1000, 64, 32, 32, device=dev).contiguous(memory_format=torch.channels_last)
    r = torch.randn_like(x)
    y = torch.empty_like(x)
    consts = torch.cat([torch.randn(64, device=dev), torch.rand(64, device=dev) + 0.5,
                        torch.rand(64, device=dev) + 0.5, torch.randn(64, device=dev)])

    def step(ea=None, eb=None):
        if ea is not None:
            ea.record()
        _native.bn_act_exact_nhwc(x, consts, residual=r, relu=True, out=y)
        if eb is not None:
            eb.record()

    _, kms = timed_launches(step, max(10, args.steps), 3, warm_s=COMPONENT_WARM_S)
    nbytes = x.numel() * 12
    del x, r, y
    return {"config": "eval BN + residual + ReLU, [1000, 64, 32, 32] fp32 channels_last",
            "roofline": roofline("dls_bn_act_exact_nhwc_f32", nbytes, kms, key="bn_act")}


# ---------------------------------------------------------- CPU baseline
def cpu_baseline(args):
    """Reference torch op sequence (servers/fed_server.py:52-65) on the host CPU."""
    from oracle.fedavg import fedavg_torch_cpu  # test infrastructure, timed only
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count()
    torch.set_num_threads(threads)
    shapes = resnet18_cifar()
    Kc = args.cpu_clients
    g = torch.Generator().manual_seed(SEED)
    clients = [{k: torch.randn(s, generator=g) * 0.05 for k, s in shapes} for _ in range(Kc)]
    n = [100 + 9 * i for i in range(Kc)]
    order = list(range(Kc))
    fedavg_torch_cpu(clients, n, order)  # warm
    reps, t0 = 0, time.perf_counter()
    while True:
        fedavg_torch_cpu(clients, n, order)
        reps += 1
        el = time.perf_counter() - t0
        if (el >= args.cpu_seconds and reps >= 2) or el >= 3 * args.cpu_seconds:
            break
    per = el / reps
    P = sum(math.prod(s) for _, s in shapes)
    shapley = cpu_shapley_eval(args, clients, n, threads)
    del clients
    model = ""
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        model = next((l.split(":", 1)[1].strip() for l in out.splitlines()
                      if l.startswith("Model name")), "")
    except Exception:
        pass
    config1 = cpu_config1(args, threads)
    return {"value": round(Kc * P * 4 / per / 1e9, 3), "unit": "GB/s", "cores": threads,
            "kind": "port",
            "sample": f"{Kc} ResNet-18 client dicts (fp32, 62 tensors), reference torch op "
                      f"sequence, {reps} reps in {el:.1f}s",
            "cpu_model": model or platform.processor(), "ms_per_aggregation": round(per * 1e3, 2),
            "components": {"shapley_evals": shapley, **cpu_components(args, threads),
                           "config1": config1}}


def cpu_shapley_eval(args, clients, n, threads):
    """Config 5b on the host: one Shapley utility evaluation the reference's way —
    get_subset_model's torch op sequence over a 25-client coalition
    (servers/fed_server.py:52-65) + ResNet-18 inference on the test set
    (servers/fed_server.py:26-32) — timed on a bounded image sample and scaled to
    the full test set (inference time is linear in the image count)."""
    from oracle.fedavg import fedavg_torch_cpu  # test infrastructure, timed only
    from distributed_learning_simulator_amd.models import ResNet18
    coal = list(range(0, len(clients), 2))[:25]
    t0 = time.perf_counter()
    model = fedavg_torch_cpu(clients, n, coal)
    t_subset = time.perf_counter() - t0
    net = ResNet18().eval()
    with torch.no_grad():
        for k, p in net.named_parameters():
            p.copy_(model[k])
    g = torch.Generator().manual_seed(SEED + 11)
    imgs = args.cpu_eval_images
    X = torch.randn(imgs, 3, 32, 32, generator=g)
    with torch.no_grad():
        net(X[:100])  # warm
        t0 = time.perf_counter()
        for i in range(0, imgs, 250):
            net(X[i:i + 250]).argmax(1)
        t_inf = (time.perf_counter() - t0) * args.eval_images / imgs
    per_eval = t_subset + t_inf
    return {"value": round(1.0 / per_eval, 4), "unit": "subset-evals/s", "cores": threads,
            "kind": "port",
            "sample": f"25-client ResNet-18 subset model (reference torch op sequence) + "
                      f"inference on {imgs} images, scaled to {args.eval_images}",
            "s_per_eval": round(per_eval, 2), "s_subset_model": round(t_subset, 3)}


def cpu_components(args, threads):
    """The reference's torch op sequences for configs 3 and 4 on the host cores
    (bounded samples; per-client rates scale linearly in K)."""
    from oracle.fedavg import fedavg_torch_cpu  # test infrastructure, timed only
    from oracle.quant import dequant_torch_cpu
    from oracle.sign import sign_vote_torch_cpu
    res = {}
    g = torch.Generator().manual_seed(SEED + 9)
    shapes = resnet18_cifar()
    P = sum(math.prod(s) for _, s in shapes)
    Ks = 20  # servers/sign_sgd_server.py:16-18 on 20 clients' fp32 sign lists
    signs = [[torch.sign(torch.randn(s, generator=g)) for _, s in shapes] for _ in range(Ks)]
    sign_vote_torch_cpu(signs)
    t0, reps = time.perf_counter(), 0
    while time.perf_counter() - t0 < args.cpu_seconds / 2 or reps < 2:
        sign_vote_torch_cpu(signs)
        reps += 1
    per = (time.perf_counter() - t0) / reps
    res["sign_vote"] = {"value": round(Ks * P * 4 / per / 1e9, 3),
                        "unit": "GB/s (fp32 sign lists, the reference's wire format)",
                        "cores": threads, "kind": "port",
                        "sample": f"{Ks} clients x ResNet-18, {reps} reps",
                        "ms_per_vote": round(per * 1e3, 2)}
    del signs
    # servers/fed_quant_server.py:25-33 per client + servers/fed_server.py:52-65
    Kq = 2
    payloads = []
    for _ in range(Kq):
        d = {}
        for name, s in vgg16():
            if len(s) >= 2:
                d[name] = (torch.randint(-128, 128, s, generator=g, dtype=torch.int8),
                           torch.rand(s[0], generator=g, dtype=torch.float64) * 1e-2,
                           torch.zeros(s[0], dtype=torch.int64))
            else:
                d[name] = torch.randn(s, generator=g)
        payloads.append(d)
    Pv = sum(math.prod(s) for _, s in vgg16())
    t0 = time.perf_counter()
    deq = [dequant_torch_cpu(p) for p in payloads]
    fedavg_torch_cpu(deq, [500] * Kq, list(range(Kq)))
    el = time.perf_counter() - t0
    res["fed_quant"] = {"value": round(Kq * Pv / el / 1e9, 3),
                        "unit": "GB/s (int8 client updates)", "cores": threads, "kind": "port",
                        "sample": f"{Kq} clients x VGG-16 dequant (channel loop) + FedAvg, 1 rep",
                        "ms_per_client": round(el / Kq * 1e3, 1)}
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--clients", type=int, default=100,
                    help="config-2 client updates: per GPU (weak) or in total (strong)")
    ap.add_argument("--scaling", choices=("weak", "strong"), default="weak",
                    help="the headline's scaling; at N > 1 the other one is a component")
    ap.add_argument("--chunks", type=int, default=3, help="all-reduce pipeline chunks (N>1)")
    ap.add_argument("--subsets", type=int, default=50)
    ap.add_argument("--evals", type=int, default=8, help="timed Shapley utility evaluations per GPU")
    ap.add_argument("--eval-images", type=int, default=10000)
    ap.add_argument("--quick", action="store_true", help="headline only (no components)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend for N>1")
    ap.add_argument("--only", default="", help="comma list: headline,fedavg_other_scaling,"
                    "fedavg_k1000,sign_vote,fed_quant,fed_quant_k1000,shapley_exact,shapley_gemm,"
                    "shapley_evals,sign_vote_sharded,fed_quant_sharded,config1")
    ap.add_argument("--cpu-clients", type=int, default=100,
                    help="CPU baseline: clients of the config-2 aggregation (full K = 100)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-eval-images", type=int, default=500)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    _native.require_gpu()
    local = local % torch.cuda.device_count()  # (gloo dry runs may oversubscribe one GPU)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)  # RCCL over xGMI
        else:  # dry runs of the N>1 path on a single-GPU box
            dist.init_process_group(args.backend)

    only = set(args.only.split(",")) if args.only else None
    want = lambda name: only is None or name in only  # noqa: E731
    value = ms = rf = None
    extra = {}
    if want("headline"):
        value, ms, rf, extra = bench_fedavg(args, dev, rank, world, args.scaling)
    components = {}
    if world > 1 and not args.quick:  # collectives: every rank takes part, no per-rank skipping
        other = "strong" if args.scaling == "weak" else "weak"
        coll = [("fedavg_other_scaling",
                 lambda *a: dict(zip(("value", "ms_per_step", "roofline", "config"),
                                     bench_fedavg(args, dev, rank, world, other)),
                                 scaling=other, unit="GB/s")),
                ("fedavg_bitexact_sharded",
                 lambda *a: bench_fedavg_bitexact_sharded(args, dev, world, rank)),
                ("sign_vote_sharded", lambda *a: bench_sign_sharded(args, dev, world, rank)),
                ("fed_quant_sharded", lambda *a: bench_quant_sharded(args, dev, world, rank)),
                ("shapley_evals", lambda *a: bench_shapley_evals(args, dev, world, rank))]
        for name, fn in coll:
            if not want(name):
                continue
            components[name] = fn()
            if rank == 0:
                log(name, json.dumps(components[name]))
            torch.cuda.empty_cache()
    if not args.quick and rank == 0:
        local_parts = [("fedavg_k1000", bench_fedavg_k1000), ("sign_vote", bench_sign),
                       ("fed_quant", bench_quant), ("fed_quant_k1000", bench_quant_k1000),
                       ("shapley_exact", bench_shapley_exact), ("shapley_gemm", bench_shapley_gemm),
                       ("config1", bench_config1)]
        if world == 1:
            local_parts.append(("shapley_evals", bench_shapley_evals))
        for name, fn in local_parts:
            if not want(name):
                continue
            try:
                components[name] = fn(args, dev)
                log(name, json.dumps(components[name]))
            except Exception as e:  # report, never hide
                components[name] = {"error": repr(e)}
            torch.cuda.empty_cache()
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and only is None:
        cpu = cpu_baseline(args)
    if world > 1:
        dist.barrier()
    if rank == 0:
        total_clients = extra.get("clients_total", args.clients)
        line = {
            # BASELINE.json's metric; `value` is its first part (client-update GB/s),
            # the second part (Shapley subset-evals/s) is `shapley_subset_evals_per_s`
            "metric": "client-update GB/s aggregated per FL round + Shapley subset-evals/sec",
            "value": round(value, 2) if value is not None else None, "unit": "GB/s",
            "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 4) if ms is not None else None,
            "higher_is_better": True,
            "scaling": args.scaling, "vs_baseline": None, "dtype": "fp32", "data": "synthetic",
            "config": {"workload": f"FedAvg aggregation of {total_clients} synthetic ResNet-18 "
                                   f"(11.2M-param fp32) client updates "
                                   f"({'per GPU' if args.scaling == 'weak' else 'in total'}), "
                                   "bit-exact reference order",
                       "parallelism": f"clients sharded over {world} GPU(s) + RCCL all-reduce",
                       **extra},
            "roofline": rf, "cpu_baseline": cpu,
            "shapley_subset_evals_per_s": (components.get("shapley_evals") or {}).get("value"),
            "components": components,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
