#!/bin/bash
# HBM bytes of the sign vote per variant library (tools/_variants/libdls_<v>.so):
# FETCH_SIZE and WRITE_SIZE passes over 3 calls of tools/ab_bench.py's vote_sign
# workload (1000 ResNet-18 clients), plus the L2 request counters named in VERDICT r05.
#   tools/vote_pmc.sh <tag> <variant> [<variant> ...]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; shift
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
    for C in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCP_TCC_READ_REQ_sum TCC_HIT_sum"; do
        D="$(mktemp -d /tmp/votepmc.XXXXXX)"
        n=$(echo $C | cut -d' ' -f1)
        timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$D" -o run -- \
            python3 "$ROOT/tools/ab_bench.py" --workloads vote_sign --only-run --launches 3 --variants "$v" \
            > "$OUT/${v}_$n.log" 2>&1 || { echo "pass $v $C failed"; tail -3 "$OUT/${v}_$n.log"; rm -rf "$D"; continue; }
        f="$D/run_counter_collection.csv"
        [ -f "$f" ] && { head -1 "$f"; grep 'dls::' "$f" || true; } > "$OUT/${v}_$n.csv"
        rm -rf "$D"
    done
done
ls "$OUT"
