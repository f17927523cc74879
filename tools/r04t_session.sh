#!/bin/bash
# Round-4 session t (GPU box): FMA mode with every lane-tile width in one launch
# (qany) vs one launch per width (qsep): quant GPU tests on the in-tree build
# (qany), then same-process A/B, outputs checked bit-identical.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/r04t"
mkdir -p "$OUT"
step() {  # $1 = log name, rest = command
    local log="$OUT/$1"; shift
    "$@" > "$log" 2>&1
    local rc=$?
    echo "== $(basename "$log") rc=$rc"; tail -8 "$log"
    [ $rc -eq 0 ] || exit $rc
}
step pytest_quant.txt timeout -k 10 600 python -u -m pytest tests/test_gpu_quant.py tests/test_gpu_simulator.py -x -v --timeout 240 --timeout-method thread -p no:cacheprovider
step ab_quant.txt timeout -k 10 500 python -u tools/ab_bench.py --workloads quant_r18_fma,quant_fma,quant_r18 --check --rounds 9
echo "session done"
