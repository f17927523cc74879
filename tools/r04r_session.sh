#!/bin/bash
# Round-4 session r (GPU box): utility inference on the NCHW deterministic path:
# inference tests, then bench.py's shapley_evals component.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/r04r
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_infer.py -x -v --timeout 240 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest_infer.txt" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|passed|failed" "$OUT/pytest_infer.txt" | tail -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --only shapley_evals --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.log"
rc=$?; echo "bench rc=$rc"; grep -v amdgpu.ids "$OUT/bench.log" | cut -c1-1500
exit $rc
