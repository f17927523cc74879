#!/bin/bash
# Round-4 probe session (GPU box): VALU issue calibration, sign-vote wave-layout
# A/B, fed_quant FMA mode and the stream / L2-resident / combined clock probe.
# Every GPU step has its own time limit; the first failure ends the session.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/r04a"
mkdir -p "$OUT"
step() {  # $1 = log name, rest = command
    local log="$OUT/$1"; shift
    "$@" > "$log" 2>&1
    local rc=$?
    echo "== $(basename "$log") rc=$rc"; tail -40 "$log"
    [ $rc -eq 0 ] || exit $rc
}
step valu_issue.txt timeout -k 10 120 "$ROOT/tools/_valu_issue_probe"
step ab_vote.txt env DLS_VARIANTS="$ROOT/tools/_variants/vote" timeout -k 10 300 \
    python -u tools/ab_bench.py --workloads vote_sign,vote --check --rounds 7
step ab_quant.txt env DLS_VARIANTS="$ROOT/tools/_variants/quant" timeout -k 10 400 \
    python -u tools/ab_bench.py --workloads quant_r18,quant_r18_fma,quant_r18_k5000,quant_r18_k5000_fma,quant_r18_k5000_l2 --rounds 5
step ab_union.txt env DLS_VARIANTS="$ROOT/tools/_variants/union" timeout -k 10 300 \
    python -u tools/ab_bench.py --workloads union --check --rounds 7
cd /tmp && export TMPDIR=/tmp
# the valu probe under the SQ counters (each dispatch its own row)
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    --output-format csv -d /tmp/vp -o run -- "$ROOT/tools/_valu_issue_probe" > "$OUT/valu_pmc.log" 2>&1 || exit $?
cp /tmp/vp/run_counter_collection.csv "$OUT/valu_pmc.csv"
# K = 5000 fed_quant dispatches (>= 10 ms): stream-only / L2-resident arithmetic /
# combined / FMA mode: kernel durations, then one SQ + GRBM pass each
for spec in stream:qstream:quant_r18_k5000 combined:qbase:quant_r18_k5000 l2:qbase:quant_r18_k5000_l2 fma:qbase:quant_r18_k5000_fma; do
    IFS=: read -r name lib wl <<< "$spec"
    mkdir -p "/tmp/lib_$name" && cp "$ROOT/tools/_variants/quant/libdls_$lib.so" "/tmp/lib_$name/"
    DLS_VARIANTS="/tmp/lib_$name" timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "/tmp/qt_$name" -o run -- \
        python3 "$ROOT/tools/ab_bench.py" --workloads "$wl" --only-run --launches 4 > "$OUT/qtrace_$name.log" 2>&1 || exit $?
    cp "/tmp/qt_$name/run_kernel_stats.csv" "$OUT/qstats_$name.csv"
    grep -E "dls::|Kernel_Name" "/tmp/qt_$name/run_kernel_trace.csv" > "$OUT/qtrace_$name.csv"
    DLS_VARIANTS="/tmp/lib_$name" timeout -s KILL 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
        --output-format csv -d "/tmp/qp_$name" -o run -- \
        python3 "$ROOT/tools/ab_bench.py" --workloads "$wl" --only-run --launches 2 > "$OUT/qpmc_$name.log" 2>&1 || exit $?
    f="/tmp/qp_$name/run_counter_collection.csv"
    { head -1 "$f"; grep 'dls::' "$f" || true; } > "$OUT/qpmc_$name.csv"
    echo "== $name done"
done
echo "session done"
