#!/bin/bash
# Evrard -n 100 step time (bench, twice) and GPU busy from a kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/e100; mkdir -p $O; export TMPDIR=/tmp
for k in 1 2; do
  timeout -k 10 200 python3 bench.py --init evrard -n 100 --steps 30 --warmup 5 > $O/b$k.json 2> $O/b$k.err || { tail -5 $O/b$k.err; exit 1; }
  echo "bench $k: $(grep -o '"ms_per_step": [0-9.]*' $O/b$k.json)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 bench.py --init evrard -n 100 --steps 8 --warmup 3 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
python3 scripts/gpu_busy.py $O/prof/run_kernel_trace.csv 8 > $O/busy.txt; head -1 $O/busy.txt
