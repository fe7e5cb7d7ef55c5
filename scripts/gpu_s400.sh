#!/bin/bash
# Sedov -n 400 steady-state kernel table (headline config)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/s400; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- \
    python3 bench.py --init sedov -n 400 --steps 4 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 scripts/gpu_busy.py $O/p/run_kernel_trace.csv 4 > $O/busy.txt; head -40 $O/busy.txt
rm -f $O/p/run_kernel_trace.csv
