#!/bin/bash
# Kernel trace of the north-star fed_quant workload (1000 x ResNet-18 int8) with the product library.
set -u
ROOT="${GRAFT_REPO_ROOT}"
mkdir -p "$ROOT/gpurun_out/trace_q18" /tmp/prodlib
cp "$ROOT/distributed_learning_simulator_amd/libdls_hip.so" /tmp/prodlib/libdls_product.so
cd /tmp && export TMPDIR=/tmp
DLS_VARIANTS=/tmp/prodlib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/tq18 -o run -- \
    python3 "$ROOT/tools/ab_bench.py" --workloads quant_r18 --only-run --launches 3 > "$ROOT/gpurun_out/trace_q18/run.log" 2>&1 || exit $?
cp /tmp/tq18/run_kernel_stats.csv "$ROOT/gpurun_out/trace_q18/"
grep -E "dls::|Kernel_Name" /tmp/tq18/run_kernel_trace.csv > "$ROOT/gpurun_out/trace_q18/kernel_trace_dls.csv"
