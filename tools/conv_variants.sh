#!/bin/bash
# Per-layer conv timings of variant libraries (tools/build_variants.py):
#   tools/conv_variants.sh <tag> <variant> [<variant> ...]
# each in its own process with DLS_HIP_LIB=tools/_variants/libdls_<variant>.so;
# output in gpurun_out/<tag>/conv_<variant>.txt.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; shift
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
for v in "$@"; do
    DLS_HIP_LIB="$ROOT/tools/_variants/libdls_$v.so" timeout -k 10 300 \
        python3 -u "$ROOT/tools/conv_probe.py" --layers-only --skip-check > "$OUT/conv_$v.txt" 2>&1 || exit $?
    echo "== $v"; grep -E "^(layer|stem)|total" "$OUT/conv_$v.txt"
done
