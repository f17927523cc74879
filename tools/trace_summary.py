#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats run: per-kernel calls / avg / min / max.

    python tools/trace_summary.py gpurun_out/prof_r01/trace/run_kernel_stats.csv [CALLS] > profiles/r01_kernel_stats.txt

With CALLS (the number of C-ABI calls the traced command made), also prints the
kernel time per call: one dls_fedavg_f32 call may launch its kernel as several
one-generation pieces, so rocprof's per-launch average is a fraction of the
per-call duration bench.py times with HIP events.

    python tools/trace_summary.py --tail N gpurun_out/prof_<tag>/trace/kernel_trace_dls.csv

per kernel, the average / min / max of its LAST N launches in the trace: the
steady state of a bench component, whose first launches (the untimed warm-up,
kernel times ramp over the first ~20-40 launches) the --stats average includes.
"""
import csv
import re
import sys


def short(name):
    m = re.search(r"(k_\w+(<[^>]*>)?)", name)
    return m.group(1) if m else name[:60]


def main(path, calls=None):
    rows = list(csv.DictReader(open(path)))
    print(f"# rocprofv3 --kernel-trace --stats summary of {path}")
    print(f"{'kernel':44s} {'calls':>6s} {'avg_us':>10s} {'min_us':>10s} {'max_us':>10s} {'share%':>7s}")
    for r in rows:
        if "dls::" not in r["Name"]:
            continue
        print(f"{short(r['Name']):44s} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:10.2f} "
              f"{float(r['MinNs']) / 1e3:10.2f} {float(r['MaxNs']) / 1e3:10.2f} "
              f"{float(r['Percentage']):7.2f}")
    if calls:
        tot = sum(float(r["TotalDurationNs"]) for r in rows if "dls::" in r["Name"])
        n = sum(int(r["Calls"]) for r in rows if "dls::" in r["Name"])
        print(f"# per C-ABI call: {n} kernel launches / {calls} calls, "
              f"{tot / calls / 1e3:.2f} us of kernel time per call")


def tail(path, n):
    by = {}
    for r in csv.DictReader(open(path)):
        if "dls::" not in r["Kernel_Name"]:
            continue
        by.setdefault(short(r["Kernel_Name"]), []).append(
            (int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    print(f"# last {n} launches per kernel of {path}")
    print(f"{'kernel':44s} {'launches':>8s} {'tail_avg_us':>11s} {'tail_min_us':>11s} {'tail_max_us':>11s}")
    for k, v in sorted(by.items(), key=lambda kv: -sum(d for _, d in kv[1])):
        d = [x for _, x in sorted(v)][-n:]
        print(f"{k:44s} {len(v):8d} {sum(d) / len(d) / 1e3:11.2f} {min(d) / 1e3:11.2f} "
              f"{max(d) / 1e3:11.2f}")


if __name__ == "__main__":
    if sys.argv[1] == "--tail":
        tail(sys.argv[3], int(sys.argv[2]))
    else:
        main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else None)
