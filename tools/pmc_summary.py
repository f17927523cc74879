#!/usr/bin/env python3
"""Summarise the per-workload rocprofv3 PMC passes of scripts_gpu_profile.sh.

Reads gpurun_out/prof_<tag>/pmc_<workload>_<COUNTER>/run_counter_collection.csv
and writes profiles/pmc_traffic.json ({workload: {...}}, read by bench.py for
roofline.traffic) plus profiles/<tag>_pmc_summary.txt.

Corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE / WRITE_SIZE are KiB; on
gfx950 FETCH_SIZE reports half the bytes of wide (16 B/lane) coalesced streaming
reads, so hbm_read = 2 * FETCH_SIZE * 1024; WRITE_SIZE reads exactly for
16-B-per-lane streaming stores.
"""
import csv
import json
import os
import re
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKLOADS = {  # workload -> [(kernel regexes summed per launch, key in pmc_traffic.json)]
    "headline": [(["k_fedavg_exact_pipe"], "headline")],
    "fedavg_k1000": [(["k_fedavg_exact_pipe"], "fedavg_k1000")],
    "sign_vote": [(["k_sign_vote"], "sign_vote"), (["k_sign_pack"], "sign_pack")],
    # one dls_dequant_fedavg call = the one-channel kernel + the general kernel
    "fed_quant": [(["k_dequant_fast", "k_dequant_general"], "fed_quant")],
    "shapley_gemm": [(["k_subset_gemm"], "shapley_gemm")],
}


def values(path, counter, kernel):
    """{full kernel name (one template instance): [value per launch]}"""
    out = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] == counter and re.search(r"\b" + kernel + r"(\b|<)", row["Kernel_Name"]):
                out.setdefault(row["Kernel_Name"], []).append(float(row["Counter_Value"]))
    return out


# C-ABI calls a workload's bench.py function makes for its --steps / --warmup
# (bench.bench_fedavg: warmup + steps; bench.bench_fedavg_k1000: 2 + max(3, steps // 4))
CALLS = {"headline": lambda s, w: s + w, "fedavg_k1000": lambda s, w: 2 + max(3, s // 4)}


def bench_calls(path, wl):
    """C-ABI calls the PMC pass of workload wl made (from its bench.py line), or None."""
    try:
        d = json.loads(open(path).read().strip().splitlines()[-1])
        return CALLS[wl](int(d["steps"]), int(d["warmup"]))
    except (OSError, ValueError, KeyError, IndexError):
        return None


def main(tag):
    base = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    res, lines = {}, []
    for wl, kernels in WORKLOADS.items():
        for names, key in kernels:
            fm = wm = 0.0
            nl = 0
            kernel = "+".join(names)
            try:
                for name in names:
                    f = values(os.path.join(base, f"pmc_{wl}_FETCH_SIZE",
                                            "run_counter_collection.csv"), "FETCH_SIZE", name)
                    w = values(os.path.join(base, f"pmc_{wl}_WRITE_SIZE",
                                            "run_counter_collection.csv"), "WRITE_SIZE", name)
                    calls = bench_calls(os.path.join(base, f"pmc_{wl}_FETCH_SIZE.json"), wl)
                    for inst in f.keys() & w.keys():
                        if calls and len(f[inst]) % calls == 0 and len(w[inst]) % calls == 0:
                            # one C-ABI call may launch an instance several times
                            # (FedAvg's one-generation pieces): bytes per call
                            fm += sum(f[inst]) / calls
                            wm += sum(w[inst]) / calls
                            nl = max(nl, calls)
                        else:  # every instance (e.g. k_dequant_fast<4..1>) once per call
                            fm += statistics.median(f[inst])
                            wm += statistics.median(w[inst])
                            nl = max(nl, len(f[inst]))
            except OSError:
                continue
            if not nl:
                continue
            rd, wr = 2.0 * fm * 1024.0, wm * 1024.0
            res[key] = {"kernel": kernel, "fetch_size_kib": fm, "write_size_kib": wm,
                        "hbm_read_bytes": rd, "hbm_write_bytes": wr,
                        "hbm_bytes_per_launch": rd + wr, "launches": nl}
            lines.append(f"{key:14s} {kernel:36s} FETCH_SIZE {fm:12.0f} KiB (x2 -> {rd / 1e9:8.3f} GB) "
                         f"WRITE_SIZE {wm:11.0f} KiB ({wr / 1e9:7.3f} GB) total "
                         f"{(rd + wr) / 1e9:8.3f} GB/call  [{nl} calls]")
    with open(os.path.join(ROOT, "profiles", "pmc_traffic.json"), "w") as fh:
        json.dump(res, fh, indent=1)
    with open(os.path.join(ROOT, "profiles", f"{tag}_pmc_summary.txt"), "w") as fh:
        fh.write(f"# rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, one pass per counter per workload ({tag})\n")
        fh.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
