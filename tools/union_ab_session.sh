#!/bin/bash
# GPU parity suite on the product library, then an interleaved A/B of the
# tools/_variants libraries on the union workload and SQ counters of the product's.
set -u
cd "${GRAFT_REPO_ROOT}"
R=$PWD
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head -20; tail -2 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u tools/ab_bench.py --workloads union,bn_act --rounds 5 > gpurun_out/ab_union.log 2>&1 || exit $?
cat gpurun_out/ab_union.log
mkdir -p /tmp/prodlib && cp distributed_learning_simulator_amd/libdls_hip.so /tmp/prodlib/libdls_product.so
DLS_VARIANTS=/tmp/prodlib bash scripts_gpu_pmc.sh union u_prod \
    "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" || exit $?
