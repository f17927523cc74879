#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) per dls kernel.

Reads gpurun_out/prof_<tag>/pmc_<COUNTER>/run_counter_collection.csv and writes
profiles/pmc_traffic.json (read by bench.py for roofline.traffic) and a
human-readable profiles/<tag>_pmc_summary.txt.

Corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reports half the bytes of wide (16 B/lane) coalesced
streaming reads, so hbm_read = 2 * FETCH_SIZE * 1024; WRITE_SIZE reads exactly
for 16-B-per-lane streaming stores.
"""
import csv
import json
import os
import re
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

KERNELS = {
    "k_fedavg_exact": "dls_fedavg_f32",
    "k_fedavg_fma": "dls_fedavg_f32_fma",
    "k_sign_vote": "dls_sign_vote",
    "k_sign_pack": "dls_sign_pack_f32",
    "k_dequant_fedavg": "dls_dequant_fedavg",
    "k_subset_gemm": "dls_subset_gemm_f32",
    "k_subset_exact": "dls_subset_fedavg_f32",
}


def kernel_key(name):
    for k, v in KERNELS.items():
        if re.search(r"\b" + k + r"\b", name):
            return v
    return None


def read(path, counter):
    vals = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            k = kernel_key(row["Kernel_Name"])
            if k:
                vals.setdefault(k, []).append(float(row["Counter_Value"]))
    return vals


def main(tag):
    base = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    fetch = read(os.path.join(base, "pmc_FETCH_SIZE", "run_counter_collection.csv"), "FETCH_SIZE")
    write = read(os.path.join(base, "pmc_WRITE_SIZE", "run_counter_collection.csv"), "WRITE_SIZE")
    out, lines = {}, []
    for k in sorted(set(fetch) | set(write)):
        f = statistics.median(fetch.get(k, [0.0]))
        w = statistics.median(write.get(k, [0.0]))
        rd = 2.0 * f * 1024.0
        wr = w * 1024.0
        out[k] = {"fetch_size_kib": f, "write_size_kib": w, "hbm_read_bytes": rd,
                  "hbm_write_bytes": wr, "hbm_bytes_per_launch": rd + wr,
                  "launches": len(fetch.get(k, []))}
        lines.append(f"{k:28s} FETCH_SIZE {f:14.0f} KiB (x2 gfx950 -> {rd / 1e9:8.3f} GB)  "
                     f"WRITE_SIZE {w:12.0f} KiB ({wr / 1e9:7.3f} GB)  total {(rd + wr) / 1e9:8.3f} GB")
    with open(os.path.join(ROOT, "profiles", "pmc_traffic.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    with open(os.path.join(ROOT, "profiles", f"{tag}_pmc_summary.txt"), "w") as fh:
        fh.write("# rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), median per launch\n")
        fh.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
