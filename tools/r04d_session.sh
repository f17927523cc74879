#!/bin/bash
# Round-4 session d: clients per batch on the lane tiles (in-flight depth), exact / FMA
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/r04d"
mkdir -p "$OUT"
DLS_VARIANTS="$ROOT/tools/_variants/quant" timeout -k 10 500 python -u tools/ab_bench.py \
    --workloads quant_r18_fma,quant_r18,quant_r18_l1_fma,quant_r18_l1,quant --rounds 5 > "$OUT/ab_depth.txt" 2>&1
rc=$?; echo "ab rc=$rc"; grep -v "^union" "$OUT/ab_depth.txt"
exit $rc
