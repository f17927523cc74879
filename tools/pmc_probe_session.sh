#!/bin/bash
# Extra rocprofv3 counter passes (diagnostics for DESIGN §10): TA/TD busy on the
# north-star fed_quant workload, LDS activity on the union kernel.
set -u
ROOT="${GRAFT_REPO_ROOT}"
OUT="$ROOT/gpurun_out/pmc_probe"
mkdir -p "$OUT" /tmp/prodlib
cp "$ROOT/distributed_learning_simulator_amd/libdls_hip.so" /tmp/prodlib/libdls_product.so
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1
pass() {  # $1 = name, $2 = workload, $3 = counters
    DLS_VARIANTS=/tmp/prodlib timeout -s KILL 90 rocprofv3 --pmc $3 --output-format csv -d "/tmp/pp_$1" -o run -- \
        python3 "$ROOT/tools/ab_bench.py" --workloads "$2" --only-run --launches 3 > "$OUT/$1.log" 2>&1
    rc=$?
    f="/tmp/pp_$1/run_counter_collection.csv"
    if [ -f "$f" ]; then { head -1 "$f"; grep 'dls::' "$f" || true; } > "$OUT/$1.csv"; fi
    return $rc
}
pass fedavg_td fedavg "TD_TD_BUSY_sum TA_TA_BUSY_sum GRBM_GUI_ACTIVE" &&
pass quant_td quant "TD_TD_BUSY_sum TA_TA_BUSY_sum GRBM_GUI_ACTIVE" &&
pass vote_td vote_sign "TD_TD_BUSY_sum TA_TA_BUSY_sum GRBM_GUI_ACTIVE"
echo "rc=$?"
