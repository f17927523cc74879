#!/usr/bin/env python3
"""Summarise tools/conv_pmc.sh pass 1 (SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT
SQ_WAIT_INST_LDS): per (kernel, grid) the medians over its dispatches of
MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8) and the
wait / active fractions of SQ_WAVE_CYCLES.
    python tools/conv_pmc_summary.py gpurun_out/<tag>/pmc_1.csv"""
import collections
import csv
import re
import statistics
import sys

rows = collections.defaultdict(dict)
for r in csv.DictReader(open(sys.argv[1])):
    k = re.sub(r"\(.*", "", r["Kernel_Name"].replace("void ", "").replace("dls::(anonymous namespace)::", ""))
    rows[(k, int(r["Grid_Size"]), r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
per = collections.defaultdict(list)
for (k, grid, _), c in rows.items():
    if "GRBM_GUI_ACTIVE" not in c or not c.get("SQ_WAVE_CYCLES"):
        continue
    wc = c["SQ_WAVE_CYCLES"]
    per[(k, grid)].append((c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (1024 * c["GRBM_GUI_ACTIVE"] / 8),
                           c.get("SQ_WAIT_ANY", 0.0) / wc, c.get("SQ_WAIT_INST_ANY", 0.0) / wc,
                           c.get("SQ_ACTIVE_INST_ANY", 0.0) / wc, c.get("SQ_WAIT_INST_LDS", 0.0) / wc))
for (k, grid), v in sorted(per.items()):
    m = [statistics.median(x[i] for x in v) for i in range(5)]
    print(f"{k:34s} grid {grid:8d} n {len(v):3d}  MFMA busy {m[0]:.3f}  WAIT_ANY {m[1]:.3f}  "
          f"WAIT_INST_ANY {m[2]:.3f}  ACTIVE_ANY {m[3]:.3f}  WAIT_INST_LDS {m[4]:.3f}")
