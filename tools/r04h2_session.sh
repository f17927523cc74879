#!/bin/bash
# Round-4 profile part 2: PMC passes of the fed_quant / Shapley / batch-norm workloads
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p gpurun_out
PROFILE_PARTS=pmc timeout -k 10 1000 bash scripts_gpu_profile.sh r04 "quant quant_fma quant_r18 quant_r18_fma union gemm bn_act" >> gpurun_out/r04h2.log 2>&1
rc=$?; echo "pmc rc=$rc"; exit $rc
