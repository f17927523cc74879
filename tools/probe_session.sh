#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/eval_probe.py --fused > gpurun_out/eval_probe.log 2>&1; echo "eval probe rc=$?"; cat gpurun_out/eval_probe.log
mkdir -p /tmp/prodlib && cp distributed_learning_simulator_amd/libdls_hip.so /tmp/prodlib/libdls_product.so
DLS_VARIANTS=/tmp/prodlib timeout -k 10 300 bash scripts_gpu_pmc.sh quant_r18 q18 || exit $?
