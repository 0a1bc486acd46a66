#!/bin/bash
# gpurun, re-submitted while the pool has no free box (exit code 3: nothing ran, nothing was
# charged); any other outcome -- success, a failing command, a refusal -- is final.
#   bash scripts/gpurun_wait.sh LOG TIMEOUT -- CMD...
LOG=$1
TO=$2
shift 3
for attempt in $(seq 1 12); do
    /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > "$LOG" 2>&1
    rc=$?
    [ $rc -ne 3 ] && break
    sleep 150
done
echo "rc=$rc" >> "$LOG"
