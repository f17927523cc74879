#!/bin/bash
# Round-4 session j (GPU box): union-kernel client-major walk A/B (tools/_variants
# ubase / ucm, outputs checked bit-identical) and the HBM stream-ceiling probe.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/r04j"
mkdir -p "$OUT"
step() {  # $1 = log name, rest = command
    local log="$OUT/$1"; shift
    "$@" > "$log" 2>&1
    local rc=$?
    echo "== $(basename "$log") rc=$rc"; tail -30 "$log"
    [ $rc -eq 0 ] || exit $rc
}
step ab_union.txt timeout -k 10 300 python -u tools/ab_bench.py --workloads union --check --rounds 7
step stream_probe.txt timeout -k 10 180 "$ROOT/tools/_stream_probe"
echo "session done"
