#!/bin/bash
# Round-4 session l (GPU box): fed_quant lane-kernel skeleton bisection
# (q0 product, q1 stream-only, q2 + no scale staging, q3 + no v_readlane addressing).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/r04l"
mkdir -p "$OUT"
timeout -k 10 400 python -u tools/ab_bench.py --workloads quant_r18 --rounds 7 > "$OUT/ab_quant.txt" 2>&1
rc=$?
tail -5 "$OUT/ab_quant.txt"
exit $rc
