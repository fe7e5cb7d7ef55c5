#!/bin/bash
# full GPU test suite (CLI now runs the bench step), Evrard -n 200 steady-state kernel table and gravity statistics
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/r4g; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 scripts/grav_stats.py --init evrard -n 200 --steps 4 > $O/grav_stats.txt 2>&1 || { tail -5 $O/grav_stats.txt; exit 1; }
tail -2 $O/grav_stats.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pe200 -o run -- \
    python3 bench.py --init evrard -n 200 --steps 6 --warmup 4 > $O/pe200.log 2>&1 || { tail -5 $O/pe200.log; exit 1; }
python3 scripts/gpu_busy.py $O/pe200/run_kernel_trace.csv 6 > $O/e200_busy.txt; head -24 $O/e200_busy.txt
