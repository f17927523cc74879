#!/bin/bash
# PMC passes over tools/conv_probe.py --layers-only (per-layer conv launches):
#   tools/conv_pmc.sh <tag> "<counters pass 1>" ["<counters pass 2>" ...]
# Each pass is its own rocprofv3 run; the dls:: rows land in gpurun_out/<tag>/pmc_<n>.csv.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; shift
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
n=0
for C in "$@"; do
    n=$((n + 1))
    D="$(mktemp -d /tmp/convpmc.XXXXXX)"
    timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d "$D" -o run -- \
        python3 -u "$ROOT/tools/conv_probe.py" --layers-only --skip-check > "$OUT/pmc_$n.log" 2>&1 || exit $?
    f="$D/run_counter_collection.csv"
    [ -f "$f" ] && { head -1 "$f"; grep 'dls::' "$f" || true; } > "$OUT/pmc_$n.csv"
    rm -rf "$D"
    tail -2 "$OUT/pmc_$n.log"
done
