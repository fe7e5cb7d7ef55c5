#!/bin/bash
# Round-2 baseline on one MI355X: GPU tests, Sedov -n 400 bench, Evrard -n 200 bench, kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_gputests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/r2_gputests.log; exit 1; }
tail -3 gpurun_out/r2_gputests.log
timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 --verbose > gpurun_out/r2_bench_sedov400.log 2>&1 || exit 1
head -1 gpurun_out/r2_bench_sedov400.log
timeout -k 10 240 python -u bench.py --init evrard -n 200 --steps 10 --warmup 3 --verbose > gpurun_out/r2_bench_evrard200.log 2>&1 || exit 1
head -1 gpurun_out/r2_bench_evrard200.log
