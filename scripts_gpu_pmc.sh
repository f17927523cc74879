#!/bin/bash
# rocprofv3 passes over one tools/ab_bench.py workload (first variant library, --only-run):
# kernel trace + stats, then one PMC pass per counter group (separate runs).
#   scripts_gpu_pmc.sh <workload> <tag> "<group1 counters>" ["<group2 counters>" ...]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")" && pwd)}"
WL="$1"; TAG="$2"; shift 2
OUT="$ROOT/gpurun_out/pmc_$TAG"
RAW="$(mktemp -d /tmp/dlspmc.XXXXXX)"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$RAW/trace" -o run -- \
    python3 "$ROOT/tools/ab_bench.py" --workloads "$WL" --only-run --launches 10 > "$OUT/trace.log" 2>&1 || exit $?
cp "$RAW/trace/run_kernel_stats.csv" "$OUT/" 2>/dev/null; grep -E "dls::|Kernel_Name" "$RAW/trace/run_kernel_trace.csv" > "$OUT/kernel_trace_dls.csv" 2>/dev/null
i=0
for G in "$@"; do
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --pmc $G --output-format csv -d "$RAW/p$i" -o run -- \
        python3 "$ROOT/tools/ab_bench.py" --workloads "$WL" --only-run --launches 3 > "$OUT/p$i.log" 2>&1 || exit $?
    f="$RAW/p$i/run_counter_collection.csv"
    if [ -f "$f" ]; then { head -1 "$f"; grep 'dls::' "$f" || true; } > "$OUT/p${i}_counters.csv"; fi
done
rm -rf "$RAW"
echo "done $OUT"
