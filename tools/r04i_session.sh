#!/bin/bash
# Round-4 bench: the driver's default bench.py run (N = 1), progress to gpurun_out/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p gpurun_out/r04i
timeout -k 10 900 python -u bench.py > gpurun_out/r04i/bench.json 2> gpurun_out/r04i/bench.log
rc=$?; echo "bench rc=$rc"; cat gpurun_out/r04i/bench.json | head -c 3000; echo; tail -3 gpurun_out/r04i/bench.log
exit $rc
