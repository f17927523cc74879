#!/bin/bash
# rocprofv3 kernel + memory-copy trace of bench.py's Shapley utility evaluations
# (the tester built on host tensors, as simulator.py builds it): shows how many
# host-to-device copies of the test set the evaluations make.
#   tools/evals_trace.sh <tag>   -> gpurun_out/<tag>/evals_*
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-evals}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
D="$(mktemp -d /tmp/evtrace.XXXXXX)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$D" -o run -- \
    python3 -u "$ROOT/bench.py" --only shapley_evals --no-cpu-baseline > "$OUT/evals.json" 2> "$OUT/evals.log" || exit $?
for f in "$D"/run_memory_copy_stats.csv "$D"/run_kernel_stats.csv; do
    [ -f "$f" ] && cp "$f" "$OUT/evals_$(basename "$f")"
done
[ -f "$D/run_memory_copy_trace.csv" ] && cp "$D/run_memory_copy_trace.csv" "$OUT/evals_memory_copy_trace.csv"
rm -rf "$D"
ls -la "$OUT"
