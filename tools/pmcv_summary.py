#!/usr/bin/env python3
"""Summarise tools/pmc_variant.sh passes: per kernel, counters per C-ABI call and
the derived fractions (busy fractions over 256 CUs and GRBM_GUI_ACTIVE/8 cycles).
    python tools/pmcv_summary.py gpurun_out/pmcv_<variant>_<workload> [calls]"""
import collections
import csv
import glob
import re
import sys

d = sys.argv[1]
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 3
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in sorted(glob.glob(f"{d}/p*_counters.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("void ", "").replace("dls::(anonymous namespace)::", "")
        k = re.sub(r"\(.*", "", k)
        agg[k][r["Counter_Name"] + "@" + f[-15:-13]] += float(r["Counter_Value"]) / calls
for k, m in agg.items():
    c = {n.split("@")[0]: v for n, v in m.items()}
    grbm = {n: v for n, v in m.items() if n.startswith("GRBM")}
    out = {}
    for n, v in m.items():
        name, p = n.split("@")
        g = m.get("GRBM_GUI_ACTIVE@" + p)
        if name.startswith(("TA_", "TD_", "TCP_")) and g:
            out[name + " busy"] = v / 256 / (g / 8)
    wc = c.get("SQ_WAVE_CYCLES")
    if wc:
        out["valu_active/wave_cyc"] = c["SQ_ACTIVE_INST_VALU"] / wc
        out["wait_inst_any/wave_cyc"] = c["SQ_WAIT_INST_ANY"] / wc
        out["wait_any/wave_cyc"] = c["SQ_WAIT_ANY"] / wc
        g = [v for n, v in m.items() if n.startswith("GRBM") and "SQ_WAVES@" + n.split("@")[1] in m][0]
        out["valu_issue"] = 4 * c["SQ_ACTIVE_INST_VALU"] / (1024 * g / 8)
        out["waves_per_simd_avg"] = wc / (g / 8) / 1024 / 4 * 4
        out["insts_valu"] = c["SQ_INSTS_VALU"]
        out["grbm_cycles"] = g
    if "FETCH_SIZE" in c:
        out["fetch_bytes_x2"] = c["FETCH_SIZE"] * 2048
    print(k, {n: (round(v, 4) if v < 100 else "%.4g" % v) for n, v in out.items()})
