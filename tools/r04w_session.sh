#!/bin/bash
# Round-4 session w (GPU box): union member-loop probes (wrong outputs by design):
# u0 product, u1 no quotient (VALU per membership 6 -> 2 packed ops), u2 one LDS
# read of t per 4 members (LDS traffic / 4).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/r04w"
mkdir -p "$OUT"
timeout -k 10 400 python -u tools/ab_bench.py --workloads union --rounds 9 > "$OUT/ab_union_probe.txt" 2>&1
rc=$?
grep -E "^union" "$OUT/ab_union_probe.txt"
exit $rc
