#!/bin/bash
# retry a gpurun call only while the pool has no free box (exit 3 / transient, nothing ran)
LOG="$1"; shift
for i in $(seq 1 12); do
    timeout 2400 /usr/local/graft/bin/gpurun "$@" > "$LOG" 2>&1
    rc=$?
    if grep -q "status=transient" "$LOG" && grep -qE "nothing was charged|no free box|backing off|taken away" "$LOG"; then
        sleep 150; continue
    fi
    echo "gpurun rc=$rc (attempt $i)" >> "$LOG"
    exit $rc
done
exit 3
