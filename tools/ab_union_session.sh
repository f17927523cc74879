#!/bin/bash
# Union-kernel A/B (tools/_variants libraries), after the product library's union parity tests.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fedavg.py -k union -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_union.log 2>&1
echo "union tests rc=$?"; tail -2 gpurun_out/pytest_union.log
timeout -k 10 300 python -u tools/ab_bench.py --workloads union --rounds 7 > gpurun_out/ab_union.log 2>&1 || exit $?
cat gpurun_out/ab_union.log
