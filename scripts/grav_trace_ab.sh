#!/bin/bash
# per-kernel gravity times (rocprofv3 kernel trace, Evrard -n 200, 3 timed steps) for each HIP variant given
# ("default" = the in-tree build)
set -o pipefail
export TMPDIR=/tmp
for tag in "$@"; do
    OUT=gpurun_out/gtrace_$tag
    mkdir -p $OUT
    if [ "$tag" = default ]; then unset SPHX_HIP_VARIANT; else export SPHX_HIP_VARIANT=$tag; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
        python3 bench.py --init evrard -n 200 --steps 3 --warmup 2 > $OUT/log 2>&1 || { tail -20 $OUT/log; exit 1; }
    python3 - $OUT/run_kernel_trace.csv $tag <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
per = collections.defaultdict(list)
for r in rows:
    per[r['Kernel_Name'].split('(')[0].replace('void ', '')[-34:]].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6)
for k, v in per.items():
    if 'grav' in k or 'Spill' in k:
        print(sys.argv[2], k, ' '.join(f'{x:.2f}' for x in v))
PY
    grep -o '"ms_per_step": [0-9.]*' $OUT/log
done
