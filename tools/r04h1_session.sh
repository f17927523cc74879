#!/bin/bash
# Round-4 profile part 1: kernel traces of bench.py's kernel components, PMC passes of 4 workloads
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p gpurun_out
PROFILE_PARTS=traces timeout -k 10 500 bash scripts_gpu_profile.sh r04 >> gpurun_out/r04h1.log 2>&1 || exit $?
echo "traces done"
PROFILE_PARTS=pmc timeout -k 10 600 bash scripts_gpu_profile.sh r04 "fedavg fedavg1k vote_sign pack" >> gpurun_out/r04h1.log 2>&1
rc=$?; echo "pmc rc=$rc"; exit $rc
