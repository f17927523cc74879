#!/bin/bash
# Round-4 profile set: rocprofv3 kernel traces of bench.py + per-workload PMC passes
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
bash scripts_gpu_profile.sh r04 > gpurun_out/r04f_profile.log 2>&1
rc=$?; echo "profile rc=$rc"; tail -5 gpurun_out/r04f_profile.log
exit $rc
