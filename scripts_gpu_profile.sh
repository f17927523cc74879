#!/bin/bash
# rocprofv3 passes over bench.py (run from the repo root on the GPU box):
#   1. kernel trace + stats of the headline alone (avg duration of the dominant kernel)
#   2. kernel trace + stats of every bench workload
#   3. per workload, one PMC pass per counter (FETCH_SIZE and WRITE_SIZE cannot share
#      a pass on gfx950), so every kernel's traffic is attributed to its workload
#   4. SQ instruction / stall counters (one pass: 8 SQ + 1 GRBM)
# Raw rocprofv3 output goes to a scratch dir on the box; only the stats CSVs and the
# counter rows of this library's kernels are kept under gpurun_out/prof_<tag>/.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")" && pwd)}"
TAG="${1:-r01b}"
OUT="$ROOT/gpurun_out/prof_$TAG"
RAW="$(mktemp -d /tmp/dlsprof.XXXXXX)"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp

keep_stats() {  # $1 = pass name
    mkdir -p "$OUT/$1"
    cp "$RAW/$1/run_kernel_stats.csv" "$OUT/$1/" 2>/dev/null
    rm -rf "$RAW/$1"
}
keep_counters() {  # $1 = pass name: header + rows of dls:: kernels only
    mkdir -p "$OUT/$1"
    f="$RAW/$1/run_counter_collection.csv"
    if [ -f "$f" ]; then
        { head -1 "$f"; grep 'dls::' "$f" || true; } > "$OUT/$1/run_counter_collection.csv"
    fi
    rm -rf "$RAW/$1"
}

timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$RAW/trace_headline" -o run -- \
    python3 "$ROOT/bench.py" --steps 20 --warmup 5 --only headline > "$OUT/trace_headline.json" 2> "$OUT/trace_headline.log" || exit $?
keep_stats trace_headline
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$RAW/trace" -o run -- \
    python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --evals 2 > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.log" || exit $?
keep_stats trace
for W in headline fedavg_k1000 sign_vote fed_quant shapley_gemm; do
    for C in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d "$RAW/pmc_${W}_$C" -o run -- \
            python3 "$ROOT/bench.py" --steps 3 --warmup 1 --only $W > "$OUT/pmc_${W}_$C.json" 2> "$OUT/pmc_${W}_$C.log" || exit $?
        keep_counters "pmc_${W}_$C"
    done
done
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d "$RAW/pmc_SQ" -o run -- \
    python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --only headline,fedavg_k1000,sign_vote,fed_quant,shapley_gemm > "$OUT/pmc_SQ.json" 2> "$OUT/pmc_SQ.log" || exit $?
keep_counters pmc_SQ
rm -rf "$RAW"
echo "profiles in $OUT"
