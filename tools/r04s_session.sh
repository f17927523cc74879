#!/bin/bash
# Round-4 profile refresh of the final tree: kernel traces of bench.py's kernel
# components, PMC passes of the two workloads whose kernels changed (FMA mode).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p gpurun_out
PROFILE_PARTS=traces timeout -k 10 500 bash scripts_gpu_profile.sh r04 >> gpurun_out/r04s.log 2>&1 || exit $?
echo "traces done"
PROFILE_PARTS=pmc timeout -k 10 600 bash scripts_gpu_profile.sh r04 "quant_fma quant_r18_fma" >> gpurun_out/r04s.log 2>&1
rc=$?; echo "pmc rc=$rc"; exit $rc
