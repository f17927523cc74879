#!/bin/bash
# rocprofv3 counter passes over one tools/ab_bench.py workload for ONE variant
# library (tools/_variants/libdls_<name>.so), separate runs per counter group.
#   tools/pmc_variant.sh <variant> <workload> "<group1>" ["<group2>" ...]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
V="$1"; WL="$2"; shift 2
OUT="$ROOT/gpurun_out/pmcv_${V}_${WL}"
LIB="$(mktemp -d /tmp/dlsv.XXXXXX)"
mkdir -p "$OUT"
cp "$ROOT/tools/_variants/libdls_$V.so" "$LIB/"
cd /tmp && export TMPDIR=/tmp
i=0
for G in "$@"; do
    i=$((i + 1))
    DLS_VARIANTS="$LIB" timeout -s KILL 120 rocprofv3 --pmc $G --output-format csv -d "$LIB/p$i" -o run -- \
        python3 "$ROOT/tools/ab_bench.py" --workloads "$WL" --only-run --launches 3 > "$OUT/p$i.log" 2>&1 || exit $?
    f="$LIB/p$i/run_counter_collection.csv"
    if [ -f "$f" ]; then { head -1 "$f"; grep 'dls::' "$f" || true; } > "$OUT/p${i}_counters.csv"; fi
done
rm -rf "$LIB"
echo "done $OUT"
