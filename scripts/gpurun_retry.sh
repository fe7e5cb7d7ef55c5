#!/bin/bash
# gpurun wrapper for the development loop: retries ONLY when the infrastructure reports a transient failure
# (box never started: nothing ran, nothing charged). usage: scripts/gpurun_retry.sh OUTFILE TIMEOUT 'command'
OUT=$1; TO=$2; CMD=$3
for attempt in $(seq 1 ${RETRIES:-12}); do
    /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$OUT" 2>&1
    if grep -q "status=transient\|backing off" "$OUT"; then sleep 90; continue; fi
    break
done
