#!/bin/bash
# Round-4 end-of-round rehearsal (GPU box): the GPU test suite, smoke(), then the
# driver's default bench.py run (N = 1); logs to gpurun_out/r04i.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/r04i
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest_gpu.txt" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_gpu.txt"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.txt" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 "$OUT/smoke.txt"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.log"
rc=$?; echo "bench rc=$rc"; head -c 3000 "$OUT/bench.json"; echo; tail -3 "$OUT/bench.log"
exit $rc
