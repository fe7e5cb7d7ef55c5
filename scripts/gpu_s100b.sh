#!/bin/bash
# Sedov -n 100 GPU busy at the default leaf capacity (512 without gravity)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/s100b; mkdir -p $O; export TMPDIR=/tmp
for k in 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$k -o run -- \
      python3 bench.py --init sedov -n 100 --steps 8 --warmup 3 > $O/p$k.log 2>&1 || { tail -5 $O/p$k.log; exit 1; }
  python3 scripts/gpu_busy.py $O/p$k/run_kernel_trace.csv 8 > $O/busy$k.txt; head -1 $O/busy$k.txt
done
timeout -k 10 200 python3 bench.py --init sedov -n 100 --steps 30 --warmup 5 > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $O/b.json
