#!/bin/bash
# Round-4 session v (GPU box): FedAvg launch pieces: one-generation pieces by the
# occupancy API (f1) vs twice that many waves per launch (f2); same-process A/B,
# outputs bit-identical.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/r04v"
mkdir -p "$OUT"
timeout -k 10 400 python -u tools/ab_bench.py --workloads fedavg,fedavg1k --rounds 9 > "$OUT/ab_fedavg.txt" 2>&1
rc=$?
grep -E "^fedavg" "$OUT/ab_fedavg.txt"
exit $rc
