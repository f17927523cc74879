#!/bin/bash
# Round-4 session k (GPU box): the lane kernel's chunk-drain hypothesis (stream probe).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/r04k"
mkdir -p "$OUT"
timeout -k 10 180 "$ROOT/tools/_stream_probe" > "$OUT/stream_probe.txt" 2>&1
rc=$?
cat "$OUT/stream_probe.txt"
exit $rc
