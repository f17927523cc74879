#!/usr/bin/env python3
"""Summarise scripts_gpu_profile.sh output into profiles/.

* profiles/pmc_traffic.json: HBM bytes per C-ABI call for each bench roofline
  key (read by bench.py as roofline.traffic), from the FETCH_SIZE / WRITE_SIZE
  passes: every pass makes exactly 3 calls (tools/ab_bench.py --only-run
  --launches 3), so bytes per call = the sum over all of
  this library's kernels in the pass / 3 (one call may launch several kernels:
  FedAvg's one-generation pieces, fed_quant's tile groups).
  Corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE / WRITE_SIZE are KiB; on
  gfx950 FETCH_SIZE reports half the bytes of wide (16 B/lane) streaming reads,
  so hbm_read = 2 * FETCH_SIZE * 1024; WRITE_SIZE is exact for 16-B stores.
  With the SQ pass it also carries `valu_busy_frac`: the fraction of the
  SIMDs' issue cycles the VALU was busy, 4 * SQ_ACTIVE_INST_VALU (one count per
  VALU instruction here, = SQ_INSTS_VALU; 4 SIMD cycles per fp32 wave64
  instruction, measured: tools/valu_issue_probe.hip — integer / logic ops cost
  ~2.5, so the fraction overstates integer-heavy kernels such as the sign
  kernels) / (1024 SIMDs * GRBM_GUI_ACTIVE / 8) (GRBM_GUI_ACTIVE is
  the sum over the 8 XCDs of each dispatch's busy cycles; rocprofv3 serialises
  dispatches while counting, so kernels that run concurrently in the product
  are counted one after another here).
* profiles/<tag>_pmc_summary.txt: the same plus the SQ counter ratios.

    python tools/pmc_traffic.py <tag>
"""
import collections
import csv
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CALLS = 3
SIMDS, XCDS = 1024, 8  # MI355X: 256 CUs x 4 SIMDs, 8 XCDs
KEYS = {"fedavg": "headline", "fedavg1k": "fedavg_k1000", "vote_sign": "sign_vote",
        "pack": "sign_pack", "quant": "fed_quant", "quant_r18": "fed_quant_k1000",
        "quant_fma": "fed_quant_fma", "quant_r18_fma": "fed_quant_k1000_fma",
        "union": "shapley_exact", "gemm": "shapley_gemm", "bn_act": "bn_act"}


def sums(path):
    tot = collections.defaultdict(float)
    kernels = set()
    with open(path) as f:
        for row in csv.DictReader(f):
            tot[row["Counter_Name"]] += float(row["Counter_Value"])
            m = re.search(r"(k_\w+(<[^>]*>)?)", row["Kernel_Name"])
            kernels.add(m.group(1) if m else row["Kernel_Name"][:40])
    return tot, sorted(kernels)


def main(tag):
    base = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    out_json, lines = {}, [f"# rocprofv3 PMC passes, tag {tag}: per C-ABI call ({CALLS} calls per pass)"]
    for wl, key in KEYS.items():
        try:
            f, kern = sums(os.path.join(base, f"pmc_{wl}_FETCH_SIZE", "run_counter_collection.csv"))
            w, _ = sums(os.path.join(base, f"pmc_{wl}_WRITE_SIZE", "run_counter_collection.csv"))
        except OSError:
            continue
        rd = 2 * f["FETCH_SIZE"] * 1024 / CALLS
        wr = w["WRITE_SIZE"] * 1024 / CALLS
        out_json[key] = {"kernels": kern, "fetch_size_kib": f["FETCH_SIZE"] / CALLS,
                         "write_size_kib": w["WRITE_SIZE"] / CALLS, "hbm_read_bytes": rd,
                         "hbm_write_bytes": wr, "hbm_bytes_per_launch": rd + wr, "calls": CALLS}
        lines.append(f"{key:16s} read {rd / 1e9:8.4f} GB  write {wr / 1e9:8.4f} GB  "
                     f"total {(rd + wr) / 1e9:8.4f} GB  kernels {', '.join(kern)}")
        try:
            sq, _ = sums(os.path.join(base, f"pmc_{wl}_SQ_WAVES", "run_counter_collection.csv"))
            wc = sq.get("SQ_WAVE_CYCLES", 0) or 1
            lines.append("    SQ per call: " + ", ".join(f"{k}={v / CALLS:.4g}" for k, v in sorted(sq.items())))
            lines.append("    of SQ_WAVE_CYCLES: " + ", ".join(
                f"{k}={sq[k] / wc:.3f}" for k in ("SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY")
                if k in sq))
            out_json[key]["sq_per_call"] = {k: v / CALLS for k, v in sorted(sq.items())}
            if sq.get("GRBM_GUI_ACTIVE") and "SQ_ACTIVE_INST_VALU" in sq:
                busy = 4 * sq["SQ_ACTIVE_INST_VALU"] / (SIMDS * sq["GRBM_GUI_ACTIVE"] / XCDS)
                out_json[key]["valu_busy_frac"] = busy
                lines.append(f"    VALU issue {busy:.3f} at the fp32 cost (4 x SQ_ACTIVE_INST_VALU / (1024 x "
                             f"GRBM_GUI_ACTIVE / 8); 4 cycles per fp32 wave64 instruction, integer / "
                             f"logic forms ~2.5, so integer-heavy kernels can exceed 1: "
                             f"profiles/r04a_valu_issue.txt)")
        except OSError:
            pass
    with open(os.path.join(ROOT, "profiles", "pmc_traffic.json"), "w") as fo:
        json.dump(out_json, fo, indent=1)
    with open(os.path.join(ROOT, "profiles", f"{tag}_pmc_summary.txt"), "w") as fo:
        fo.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r02")
