#!/bin/bash
# Round-4 session g: smoke, full GPU tests, product A/B of the fed_quant modes,
# rocprofv3 kernel traces of bench.py (PMC passes: session h)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/r04g"
mkdir -p "$OUT" /tmp/prodlib
cp distributed_learning_simulator_amd/libdls_hip.so /tmp/prodlib/libdls_product.so
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" "$OUT/pytest_gpu.log" | head -20; tail -2 "$OUT/pytest_gpu.log"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
DLS_VARIANTS=/tmp/prodlib timeout -k 10 300 python -u tools/ab_bench.py \
    --workloads quant_r18,quant_r18_fma,quant_r18_l1_fma,quant,quant_fma --rounds 5 > "$OUT/ab_product.txt" 2>&1
rc=$?; echo "ab product rc=$rc"; grep -v "^union member" "$OUT/ab_product.txt"; [ $rc -eq 0 ] || exit $rc
PROFILE_PARTS=traces timeout -k 10 600 bash scripts_gpu_profile.sh r04 > "$OUT/profile_traces.log" 2>&1
rc=$?; echo "traces rc=$rc"; tail -3 "$OUT/profile_traces.log"
exit $rc
