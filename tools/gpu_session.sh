#!/bin/bash
# One parameterized GPU-box session (replaces the round-4 one-shot *_session.sh).
#
#   tools/gpu_session.sh <tag> <step> [<step> ...]
#
# Output goes to gpurun_out/<tag>/; steps run in order, each under its own time
# limit, and the session stops at the first failing step (no GPU step after a
# fault, an abort or a time limit).  Steps:
#   test:<pytest args>           python -m pytest <args> -m gpu (thread timeouts)
#   ab:<workloads>[:<rounds>]    tools/ab_bench.py over every tools/_variants lib
#   abv:<variants>:<workloads>[:<rounds>]   the same, only the named variants
#   check:<variants>:<workloads> bit-identity of the named variants' outputs
#   bench[:<bench.py args>]      python bench.py (default --steps 20 --warmup 5)
#   trace:<workloads>[:<launches>]  rocprofv3 --kernel-trace --stats of ab_bench --only-run
#   pmc:<counters>:<workloads>   one rocprofv3 --pmc pass (counters comma-separated)
#   pmcv:<variant>:<counters>:<workload>:<name>  one --pmc pass of one variant -> <name>.csv
#   py:<script> [args]           python -u <script> [args]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
export TMPDIR=/tmp
TAG="$1"
shift
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
n=0
for step in "$@"; do
    n=$((n + 1))
    kind="${step%%:*}"
    rest="${step#*:}"
    [ "$rest" = "$step" ] && rest=""
    log="$OUT/$(printf %02d $n)_$kind.txt"
    echo "== step $n: $step" | tee -a "$OUT/session.txt"
    case "$kind" in
    test)
        # shellcheck disable=SC2086
        timeout -k 10 900 python -u -m pytest $rest -m gpu -x -v --timeout 240 \
            --timeout-method thread -p no:cacheprovider > "$log" 2>&1
        rc=$?
        tail -3 "$log"
        ;;
    ab)
        wl="${rest%%:*}"
        rounds="${rest#*:}"
        [ "$rounds" = "$rest" ] && rounds=5
        timeout -k 10 900 python -u tools/ab_bench.py --workloads "$wl" --rounds "$rounds" > "$log" 2>&1
        rc=$?
        grep -E "^[a-z_0-9]+ (\{|skip)" "$log"
        ;;
    abv | check)
        var="${rest%%:*}"
        rest2="${rest#*:}"
        wl="${rest2%%:*}"
        rounds="${rest2#*:}"
        [ "$rounds" = "$rest2" ] && rounds=5
        extra=""
        [ "$kind" = check ] && extra="--check"
        timeout -k 10 900 python -u tools/ab_bench.py --variants "$var" --workloads "$wl" \
            --rounds "$rounds" $extra > "$log" 2>&1
        rc=$?
        grep -E "^[a-z_0-9]+ (\{|skip|check)" "$log"
        ;;
    bench)
        args="${rest:---steps 20 --warmup 5}"
        # shellcheck disable=SC2086
        timeout -k 10 900 python -u bench.py $args > "$log" 2>&1
        rc=$?
        tail -c 3000 "$log"
        ;;
    trace)
        wl="${rest%%:*}"
        launches="${rest#*:}"
        [ "$launches" = "$rest" ] && launches=20
        timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$n" \
            -o run -- \
            python3 -u tools/ab_bench.py --workloads "$wl" --only-run --launches "$launches" \
            > "$log" 2>&1
        rc=$?
        find "$OUT/trace_$n" -name "*kernel_stats.csv" -exec head -20 {} \; | tee -a "$log"
        ;;
    pmc)
        ctr="${rest%%:*}"
        wl="${rest#*:}"
        timeout -s KILL 300 rocprofv3 --pmc ${ctr//,/ } --output-format csv -d "$OUT/pmc_$n" -o run -- \
            python3 -u tools/ab_bench.py --workloads "$wl" --only-run --launches 5 > "$log" 2>&1
        rc=$?
        tail -3 "$log"
        ;;
    pmcv)
        # pmcv:<variant>:<counters>:<workload>:<name>  one counter pass of ONE variant
        # library, its counter rows kept as <name>.csv
        var="${rest%%:*}"; r2="${rest#*:}"
        ctr="${r2%%:*}"; r3="${r2#*:}"
        wl="${r3%%:*}"; name="${r3#*:}"
        lib="$(mktemp -d /tmp/dlsv.XXXXXX)"
        cp "$ROOT/tools/_variants/libdls_$var.so" "$lib/"
        DLS_VARIANTS="$lib" timeout -s KILL 300 rocprofv3 --pmc ${ctr//,/ } --output-format csv \
            -d "$lib/p" -o run -- python3 -u tools/ab_bench.py --workloads "$wl" --only-run \
            --launches 2 > "$log" 2>&1
        rc=$?
        f="$lib/p/run_counter_collection.csv"
        [ -f "$f" ] && { head -1 "$f"; grep 'dls::' "$f" || true; } > "$OUT/$name.csv"
        rm -rf "$lib"
        tail -2 "$log"
        ;;
    py)
        # shellcheck disable=SC2086
        timeout -k 10 900 python -u $rest > "$log" 2>&1
        rc=$?
        tail -40 "$log"
        ;;
    *)
        echo "unknown step kind: $kind"
        rc=2
        ;;
    esac
    echo "== step $n rc=$rc" | tee -a "$OUT/session.txt"
    [ $rc -eq 0 ] || exit $rc
done
