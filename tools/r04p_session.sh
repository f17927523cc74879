#!/bin/bash
# Round-4 session p (GPU box): where bench.py's shapley_evals component spends its
# time on a fresh box (phase timings to stderr; a 30 s heartbeat of the log).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/r04p
mkdir -p "$OUT"
timeout -k 10 700 python -u bench.py --only shapley_evals --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.log" &
pid=$!
while kill -0 $pid 2>/dev/null; do sleep 30; echo "[$(date +%T)] $(tail -1 "$OUT/bench.log" | cut -c1-150)"; done
wait $pid
rc=$?
echo "bench rc=$rc"; cat "$OUT/bench.log" | grep -v amdgpu.ids | cut -c1-300
exit $rc
