#!/bin/bash
# Round-4 session q (GPU box): MIOpen deterministic vs default convolutions,
# NHWC vs NCHW, ResNet-18 inference on 10k images (one process per configuration),
# and the kernels of the slow one.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/r04q
mkdir -p "$OUT"
for cfg in "nchw nondet" "nchw det" "nhwc nondet" "nhwc det"; do
    timeout -k 10 240 python -u tools/eval_det_probe.py $cfg >> "$OUT/probe.txt" 2>&1 || { echo "failed: $cfg"; cat "$OUT/probe.txt"; exit 1; }
    tail -1 "$OUT/probe.txt"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ed -o run -- \
    python3 "$ROOT/tools/eval_det_probe.py" nhwc det > "$ROOT/$OUT/trace.log" 2>&1 || exit $?
cp /tmp/ed/run_kernel_stats.csv "$ROOT/$OUT/stats_nhwc_det.csv"
head -12 "$ROOT/$OUT/stats_nhwc_det.csv" | cut -c1-200
