#!/bin/bash
# Round-4 session u (GPU box): fed_quant launch order, bulk group before (qfirst)
# or after (qlast) the side groups; same-process A/B, outputs checked bit-identical.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/r04u"
mkdir -p "$OUT"
timeout -k 10 500 python -u tools/ab_bench.py --workloads quant_r18_fma,quant_r18,quant_fma,quant --check --rounds 9 > "$OUT/ab_order.txt" 2>&1
rc=$?
grep -E "^quant" "$OUT/ab_order.txt"
exit $rc
