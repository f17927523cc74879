#!/bin/bash
# rocprofv3 passes over bench.py (run from the repo root on the GPU box):
#   1. kernel trace + stats of the headline alone (avg duration of the dominant kernel)
#   2. kernel trace + stats of everything
#   3. per workload, one PMC pass per counter (FETCH_SIZE and WRITE_SIZE cannot share
#      a pass on gfx950), so every kernel's traffic is attributed to its workload
#   4. SQ instruction / stall counters (one pass: 8 SQ + 1 GRBM)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")" && pwd)}"
TAG="${1:-r01b}"
OUT="$ROOT/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_headline" -o run -- \
    python3 "$ROOT/bench.py" --steps 20 --warmup 5 --only headline > "$OUT/trace_headline.json" 2> "$OUT/trace_headline.log" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.log" || exit $?
for W in headline fedavg_k1000 sign_vote fed_quant shapley_gemm; do
    for C in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_${W}_$C" -o run -- \
            python3 "$ROOT/bench.py" --steps 3 --warmup 1 --only $W > "$OUT/pmc_${W}_$C.json" 2> "$OUT/pmc_${W}_$C.log" || exit $?
    done
done
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_SQ" -o run -- \
    python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --evals 1 > "$OUT/pmc_SQ.json" 2> "$OUT/pmc_SQ.log" || exit $?
echo "profiles in $OUT"
