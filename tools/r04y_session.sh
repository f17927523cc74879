#!/bin/bash
# Round-4 session y (GPU box): fed_quant FMA residency: the fp32 group's clients in
# flight (16: 222 VGPRs, 12: 173, 8: 125) and bulk-first launch, so that every
# wave of the call is resident at once; same process, outputs bit-identical.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/r04y"
mkdir -p "$OUT"
timeout -k 10 500 python -u tools/ab_bench.py --workloads quant_r18_fma,quant_r18,quant_fma --check --rounds 9 > "$OUT/ab_resid.txt" 2>&1
rc=$?
grep -E "^quant" "$OUT/ab_resid.txt"
exit $rc
