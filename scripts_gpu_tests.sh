#!/bin/bash
# GPU parity tests only (optionally a -k expression).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread -p no:cacheprovider "$@" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_gpu.log | grep -vE "PASSED" | head -30; tail -3 gpurun_out/pytest_gpu.log
exit $rc
