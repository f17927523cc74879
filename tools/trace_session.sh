#!/bin/bash
# rocprofv3 evidence on one GPU box without re-running the suite: a kernel trace
# of the utility evaluation's convolutions (tools/conv_probe.py) and one of the
# default bench (stats over all launches + each kernel's last 10 launches).
#   tools/trace_session.sh <tag>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-trace}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
D="$(mktemp -d /tmp/convtrace.XXXXXX)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$D" -o run -- \
    python3 -u "$ROOT/tools/conv_probe.py" --skip-check --reps 3 > "$OUT/conv_trace.log" 2>&1 || exit $?
{ head -1 "$D/run_kernel_stats.csv"; grep "dls::" "$D/run_kernel_stats.csv" || true; } > "$OUT/conv_kernel_stats.csv"
rm -rf "$D"
echo "conv trace: $OUT/conv_kernel_stats.csv"
D2="$(mktemp -d /tmp/benchtrace.XXXXXX)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$D2" -o run -- \
    python3 -u "$ROOT/bench.py" > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.err" || exit $?
cd "$ROOT"
cp "$D2/run_kernel_stats.csv" "$OUT/kernel_stats_all.csv"
{ head -1 "$D2/run_kernel_trace.csv"; grep "dls::" "$D2/run_kernel_trace.csv" || true; } > "$D2/kernel_trace_dls.csv"
python3 tools/trace_summary.py "$OUT/kernel_stats_all.csv" > "$OUT/kernel_stats_all.txt"
python3 tools/trace_summary.py --tail 10 "$D2/kernel_trace_dls.csv" > "$OUT/kernel_tail10_all.txt"
rm -rf "$D2"
echo "bench trace: $OUT/kernel_stats_all.txt $OUT/kernel_tail10_all.txt"
