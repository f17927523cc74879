#!/usr/bin/env python3
"""Summarise the fed_quant clock / issue probes (run as a tools/gpu_session.sh "py:tools/quant_bound.py ..." step):
per kernel of each dispatch kind (stream-only, L2-resident arithmetic, combined,
FMA mode), the kernel time, the effective clock GRBM_GUI_ACTIVE / 8 / duration
(MI355X_MICROARCH.md DVFS item: valid for dispatches >= 10 ms; the K = 5000 lane
pieces run 3-4 ms each, the whole call ~10 ms), VALU and vector-memory
instructions, and the SQ wave-cycle split.

    python tools/quant_bound.py gpurun_out/r04a
"""
import collections
import csv
import os
import re
import sys


def kernel_key(name):
    m = re.search(r"(k_\w+)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:40]


def summarise(path):
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        key = (r["Dispatch_Id"], kernel_key(r["Kernel_Name"]))
        per[key][r["Counter_Name"]] = float(r["Counter_Value"])
        per[key]["dur_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    agg = collections.defaultdict(collections.Counter)
    for (_, k), v in per.items():
        agg[k]["n"] += 1
        for c, x in v.items():
            agg[k][c] += x
    return agg


def main(d):
    out = []
    for name in ("stream", "l2", "combined", "fma"):
        p = os.path.join(d, f"qpmc_{name}.csv")
        if not os.path.exists(p):
            continue
        out.append(f"== {name}")
        for k, v in sorted(summarise(p).items(), key=lambda kv: -kv[1]["dur_ns"]):
            n = v["n"]
            dur = v["dur_ns"] / n
            clk = v["GRBM_GUI_ACTIVE"] / n / 8 / dur
            wc = v["SQ_WAVE_CYCLES"] or 1
            out.append(
                f"  {k:34s} n={n:2d} {dur / 1e6:7.3f} ms/dispatch  clock {clk:4.2f} GHz  "
                f"VALU {v['SQ_INSTS_VALU'] / n:.3e}  VMEM_RD {v['SQ_INSTS_VMEM_RD'] / n:.3e}  "
                f"waves {v['SQ_WAVES'] / n:.0f}  of wave-cycles: VALU {v['SQ_ACTIVE_INST_VALU'] / wc:.3f}"
                f" wait {v['SQ_WAIT_ANY'] / wc:.3f} issue-wait {v['SQ_WAIT_INST_ANY'] / wc:.3f}")
    print("\n".join(out))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/r04a")
