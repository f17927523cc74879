#!/bin/bash
# rocprofv3 evidence for the bench line (run from the repo root on the GPU box):
#   1. kernel trace + stats of bench.py's headline (FedAvg, config 2) alone;
#   2. kernel trace + stats of every bench.py workload (no CPU baseline);
#   3. per workload, separate PMC passes for FETCH_SIZE and WRITE_SIZE (they cannot
#      share a pass on gfx950) and one of 8 SQ counters + GRBM_GUI_ACTIVE, each over exactly
#      N + 1 C-ABI calls of the product library (tools/ab_bench.py --only-run).
# Only the stats CSVs and the counter rows of this library's kernels are kept,
# under gpurun_out/prof_<tag>/; tools/pmc_traffic.py summarises them.
#   scripts_gpu_profile.sh <tag> [workloads]
# PROFILE_PARTS="traces" / "pmc" runs only that part (a gpurun call is capped at 20 min).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")" && pwd)}"
TAG="${1:-r02}"
WLS="${2:-fedavg fedavg1k vote_sign pack quant quant_fma quant_r18 quant_r18_fma union gemm bn_act}"
OUT="$ROOT/gpurun_out/prof_$TAG"
RAW="$(mktemp -d /tmp/dlsprof.XXXXXX)"
LIBDIR="$RAW/lib"
mkdir -p "$OUT" "$LIBDIR"
cp "$ROOT/distributed_learning_simulator_amd/libdls_hip.so" "$LIBDIR/libdls_product.so"
cd /tmp && export TMPDIR=/tmp
keep_stats() {  # $1 = pass name
    mkdir -p "$OUT/$1"
    cp "$RAW/$1/run_kernel_stats.csv" "$OUT/$1/" 2>/dev/null
    grep -E "dls::|Kernel_Name" "$RAW/$1/run_kernel_trace.csv" > "$OUT/$1/kernel_trace_dls.csv" 2>/dev/null
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
PARTS="${PROFILE_PARTS:-traces pmc}"
if [[ "$PARTS" == *traces* ]]; then
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$RAW/trace_headline" -o run -- \
    python3 "$ROOT/bench.py" --steps 20 --warmup 5 --only headline > "$OUT/trace_headline.json" 2> "$OUT/trace_headline.log" || exit $?
keep_stats trace_headline
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$RAW/trace" -o run -- \
    python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline \
    --only headline,fedavg_k1000,sign_vote,fed_quant,fed_quant_k1000,shapley_exact,shapley_gemm \
    > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.log" || exit $?
keep_stats trace
fi
[[ "$PARTS" == *pmc* ]] || { rm -rf "$RAW"; echo "profiles in $OUT"; exit 0; }
for W in $WLS; do
    for C in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"; do
        P="pmc_${W}_$(echo $C | cut -d' ' -f1)"
        DLS_VARIANTS="$LIBDIR" timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d "$RAW/$P" -o run -- \
            python3 "$ROOT/tools/ab_bench.py" --workloads "$W" --only-run --launches 3 > "$OUT/$P.log" 2>&1 || exit $?
        keep_counters "$P"
    done
done
rm -rf "$RAW"
echo "profiles in $OUT"
