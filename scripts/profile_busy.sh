#!/bin/bash
# Kernel trace + stats of a bench configuration and its GPU-busy fraction (scripts/gpu_busy.py).
# usage: bash scripts/profile_busy.sh TAG [bench args...]   -> gpurun_out/busy_TAG/{stats,busy.txt}
set -o pipefail
TAG=$1; shift
R=$(pwd)
OUT=$R/gpurun_out/busy_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- \
    python3 "$R/bench.py" --steps 5 --warmup 2 "$@" > "$OUT/stats.log" 2>&1 || exit $?
python3 "$R/scripts/gpu_busy.py" "$OUT/stats/run_kernel_trace.csv" 3 > "$OUT/busy.txt" && cat "$OUT/busy.txt"
