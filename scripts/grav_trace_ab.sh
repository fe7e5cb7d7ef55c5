#!/bin/bash
# per-kernel gravity times (rocprofv3 kernel trace, Evrard -n 200, 2 timed steps) for each HIP variant given
set -o pipefail
export TMPDIR=/tmp
for tag in "$@"; do
    OUT=gpurun_out/gtrace_$tag
    mkdir -p $OUT
    SPHX_HIP_VARIANT=$tag timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
        python3 bench.py --init evrard -n 200 --steps 2 --warmup 2 > $OUT/log 2>&1 || { tail -20 $OUT/log; exit 1; }
    python3 - $OUT/run_kernel_stats.csv $tag <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:8]:
    print(sys.argv[2], r['Name'][:40], r['Calls'], round(float(r['TotalDurationNs']) / 1e6 / int(r['Calls']), 3), 'ms/call')
PY
    grep -o '"ms_per_step": [0-9.]*' $OUT/log
done
