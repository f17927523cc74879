#!/bin/bash
# One GPU-box session: smoke, selected GPU tests, then a probe command.
#   tools/gpu_probe_session.sh "<pytest -k expr or empty>" "<probe command or empty>" [probe timeout s]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
if [ -n "$1" ]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread \
        -p no:cacheprovider -k "$1" > gpurun_out/pytest_gpu.log 2>&1
    rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head -20
    grep -E "config-5 utilities" gpurun_out/pytest_gpu.log | head -3
    tail -2 gpurun_out/pytest_gpu.log
    [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
if [ -n "${2:-}" ]; then
    timeout -k 10 "${3:-400}" bash -c "$2" > gpurun_out/probe.log 2>&1
    rc=$?; echo "probe rc=$rc"; cat gpurun_out/probe.log | tail -60; [ $rc -eq 0 ] || exit $rc
fi
exit 0
