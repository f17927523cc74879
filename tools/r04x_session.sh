#!/bin/bash
# Round-4 session x (GPU box): FMA lane-tile width policy (fewest tiles of <= 4
# channel rows: quant_r18_fma) vs the previous rule (quant_r18_fma_oldtab), twice
# interleaved; then the quant GPU tests on the new tables.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/r04x"
mkdir -p "$OUT"
timeout -k 10 400 python -u tools/ab_bench.py --workloads quant_r18_fma,quant_r18_fma_oldtab,quant_r18_fma,quant_r18_fma_oldtab --rounds 9 > "$OUT/ab_tab.txt" 2>&1
rc=$?; grep -E "^quant" "$OUT/ab_tab.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_quant.py -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_quant.txt" 2>&1
rc=$?; tail -2 "$OUT/pytest_quant.txt"; exit $rc
