#!/bin/bash
# Round-end rehearsal on one GPU box: the GPU suite, smoke(), the default bench,
# and a rocprofv3 kernel trace of the utility evaluation's convolutions.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG="${1:-final}"
tools/gpu_session.sh "$TAG" "test:tests" "py:tools/smoke_run.py" "bench" || exit $?
OUT="$ROOT/gpurun_out/$TAG"
D="$(mktemp -d /tmp/convtrace.XXXXXX)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$D" -o run -- \
    python3 -u "$ROOT/tools/conv_probe.py" --skip-check --reps 3 > "$OUT/conv_trace.log" 2>&1 || exit $?
{ head -1 "$D/run_kernel_stats.csv"; grep "dls::" "$D/run_kernel_stats.csv" || true; } > "$OUT/conv_kernel_stats.csv"
rm -rf "$D"
echo "conv trace: $OUT/conv_kernel_stats.csv"
