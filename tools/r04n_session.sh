#!/bin/bash
# Round-4 session n (GPU box): kernel timeline of the fed_quant FMA and exact calls.
# tools/_variants holds libdls_qnew.so (this tree) and libdls_qold.so; --only-run
# launches the first, qnew.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/r04n"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/qn -o run -- \
    python3 "$ROOT/tools/ab_bench.py" --workloads quant_r18_fma,quant_r18 --only-run --launches 6 > "$OUT/trace.log" 2>&1 || exit $?
cp /tmp/qn/run_kernel_stats.csv "$OUT/stats.csv"
grep -E "dls::|Kernel_Name" /tmp/qn/run_kernel_trace.csv > "$OUT/trace.csv"
echo done
