#!/bin/bash
# Round-4 session o (GPU box): fed_quant side-group tile sizes (fp32 / small int
# tiles of 256 vs 128 vs 64 elements), FMA and exact, 1000 x ResNet-18.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/r04o"
mkdir -p "$OUT"
timeout -k 10 500 python -u tools/ab_bench.py --rounds 7 --workloads \
    quant_r18_fma,quant_r18_fma_f64,quant_r18_fma_f64s64,quant_r18_fma_f128s128,quant_r18_fma,quant_r18,quant_r18_f64,quant_r18_f64s64,quant_r18_f128s128,quant_r18 \
    > "$OUT/ab_tiles.txt" 2>&1
rc=$?
grep -E "^quant" "$OUT/ab_tiles.txt"
exit $rc
