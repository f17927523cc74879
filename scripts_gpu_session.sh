#!/bin/bash
# One GPU-box session: smoke, GPU parity tests, optional A/B probe, optional bench.
# Every GPU step has its own time limit; the first failure ends the session.
#   scripts_gpu_session.sh [--tests "<pytest -k expr>"|--no-tests] [--ab "<workloads>"] [--bench "<bench args>"]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
mkdir -p gpurun_out
TESTS="all"; AB=""; BENCH=""
while [ $# -gt 0 ]; do
    case "$1" in
        --tests) TESTS="$2"; shift 2 ;;
        --no-tests) TESTS=""; shift ;;
        --ab) AB="$2"; shift 2 ;;
        --bench) BENCH="$2"; shift 2 ;;
        *) echo "unknown arg $1"; exit 2 ;;
    esac
done
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
if [ -n "$TESTS" ]; then
    K=(); [ "$TESTS" != "all" ] && K=(-k "$TESTS")
    timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread \
        -p no:cacheprovider "${K[@]}" > gpurun_out/pytest_gpu.log 2>&1
    rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head -20
    tail -2 gpurun_out/pytest_gpu.log
    [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
if [ -n "$AB" ]; then
    timeout -k 10 400 python -u tools/ab_bench.py --workloads "$AB" --rounds 5 > gpurun_out/ab.log 2>&1
    rc=$?; echo "ab rc=$rc"; cat gpurun_out/ab.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$BENCH" ]; then
    timeout -k 10 600 python -u bench.py $BENCH > gpurun_out/bench.json 2> gpurun_out/bench.log
    rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -5 gpurun_out/bench.log
    [ $rc -eq 0 ] || exit $rc
fi
exit 0
