#!/bin/bash
# Round-4 session b: smoke, the full GPU test suite, then the fed_quant lane-tiling
# / FMA-mode A/B (store tiling adaptive vs 1 KiB; exact, FMA, stream-only probe).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/r04b"
mkdir -p "$OUT"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1200 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" "$OUT/pytest_gpu.log" | head -20; tail -2 "$OUT/pytest_gpu.log"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
DLS_VARIANTS="$ROOT/tools/_variants/quant" timeout -k 10 400 python -u tools/ab_bench.py \
    --workloads quant_r18,quant_r18_l1,quant_r18_fma,quant_r18_l1_fma,quant --rounds 5 > "$OUT/ab_quant.txt" 2>&1
rc=$?; echo "ab rc=$rc"; grep -v "^union" "$OUT/ab_quant.txt"
exit $rc
