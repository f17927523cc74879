#!/bin/bash
# Round-4 PMC passes (FETCH_SIZE, WRITE_SIZE, SQ) for the given workloads
#   tools/r04h_pmc.sh "<workloads>"
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p gpurun_out
PROFILE_PARTS=pmc timeout -k 10 1100 bash scripts_gpu_profile.sh r04 "$1" > "gpurun_out/r04h_pmc_$(echo $1 | tr ' ' '_').log" 2>&1
rc=$?; echo "pmc rc=$rc"; ls gpurun_out/prof_r04 | head -50
exit $rc
