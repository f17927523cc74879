#!/bin/bash
# rocprofv3 passes over bench.py: kernel trace + stats, then one PMC pass per
# counter (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")" && pwd)}"
TAG="${1:-r01}"
OUT="$ROOT/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.log" || exit $?
for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_$C" -o run -- \
        python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/pmc_$C.json" 2> "$OUT/pmc_$C.log" || exit $?
done
echo "profiles in $OUT"
# SQ instruction / stall counters (one pass: 8 SQ + GRBM)
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_SQ" -o run -- \
    python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --evals 1 > "$OUT/pmc_SQ.json" 2> "$OUT/pmc_SQ.log" || exit $?
echo "sq counters done"
