#!/bin/bash
# bucket 128 default (no gravity): full GPU suite, Noh -n 300 kernels, default bench, Turbulence -n 600
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/b128; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pnoh -o run -- \
    python3 bench.py --init noh -n 300 --steps 4 --warmup 3 > $O/noh300.json 2> $O/noh300.err || { tail -5 $O/noh300.err; exit 1; }
python3 scripts/gpu_busy.py $O/pnoh/run_kernel_trace.csv 4 > $O/noh300_busy.txt; head -12 $O/noh300_busy.txt
rm -f $O/pnoh/run_kernel_trace.csv
timeout -k 10 400 python3 bench.py --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"evrard_ms_per_step": [0-9.]*\|"peak_mem_gib": [0-9.]*' $O/bench.json | tr '\n' ' '; echo
timeout -k 10 500 python3 bench.py --init turbulence -n 600 --steps 3 --warmup 2 > $O/turb600.json 2> $O/turb600.err || { tail -5 $O/turb600.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"peak_mem_gib": [0-9.]*' $O/turb600.json | tr '\n' ' '
