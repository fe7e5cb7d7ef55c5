#!/bin/bash
# round-4 numbers: Sedov -n 100 GPU busy (kernel trace), Turbulence -n 600 and Noh -n 300 step times
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/r4final; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/s100 -o run -- \
    python3 bench.py --init sedov -n 100 --steps 8 --warmup 3 > $O/s100.log 2>&1 || { tail -5 $O/s100.log; exit 1; }
python3 scripts/gpu_busy.py $O/s100/run_kernel_trace.csv 8 > $O/s100_busy.txt; head -1 $O/s100_busy.txt
for c in "noh 300" "turbulence 600"; do
  set -- $c
  timeout -k 10 400 python3 bench.py --init $1 -n $2 --steps 4 --warmup 2 > $O/$1$2.json 2> $O/$1$2.err || { tail -5 $O/$1$2.err; exit 1; }
  echo "$c: $(grep -o '"ms_per_step": [0-9.]*\|"peak_mem_gib": [0-9.]*' $O/$1$2.json | tr '\n' ' ')"
done
