#!/bin/bash
# Turbulence -n 600 (225 M particles) kernel table, steady state
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/turb600; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- \
    python3 bench.py --init turbulence -n 600 --steps 3 --warmup 2 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 scripts/gpu_busy.py $O/p/run_kernel_trace.csv 2 > $O/busy.txt; head -22 $O/busy.txt
rm -f $O/p/run_kernel_trace.csv
