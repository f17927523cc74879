#!/bin/bash
# Union-kernel variant probe: the new inference tests, an interleaved A/B of the
# tools/_variants libraries on the union workload, then SQ counter passes per variant.
set -u
cd "${GRAFT_REPO_ROOT}"
R=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_infer.py -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_infer.log 2>&1
echo "infer tests rc=$?"; tail -3 gpurun_out/pytest_infer.log
timeout -k 10 300 python -u tools/ab_bench.py --workloads union --rounds 5 > gpurun_out/ab_union.log 2>&1 || exit $?
cat gpurun_out/ab_union.log
for v in lds reg2 reg4 sel4; do
  DLS_VARIANTS=$R/tools/_variants/only_$v bash scripts_gpu_pmc.sh union u_$v \
    "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY" \
    "SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_IFETCH SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_LDS" || exit $?
done
