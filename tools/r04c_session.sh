#!/bin/bash
# Round-4 session c: slab-major dequant layout emulation (exact / FMA / stream-only)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/r04c"
mkdir -p "$OUT"
DLS_VARIANTS="$ROOT/tools/_variants/quant" timeout -k 10 500 python -u tools/ab_bench.py \
    --workloads quant_r18_l1,quant_r18_l1_fma,quant_r18_fma,quant_r18_slab,quant_r18_slab_fma,quant_r18_slab4,quant_r18_slab4_fma \
    --rounds 5 > "$OUT/ab_slab.txt" 2>&1
rc=$?; echo "ab rc=$rc"; grep -v "^union" "$OUT/ab_slab.txt"
exit $rc
