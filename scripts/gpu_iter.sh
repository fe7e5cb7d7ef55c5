#!/bin/bash
# Iteration pass on one MI355X: selected GPU tests, then Sedov -n 400 and Evrard -n 200 benches (--verbose substeps).
# usage: bash scripts/gpu_iter.sh TAG [pytest targets...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-iter}; shift
TESTS=${@:-tests}
timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 --verbose > gpurun_out/${TAG}_sedov400.log 2>&1 || { tail -20 gpurun_out/${TAG}_sedov400.log; exit 1; }
grep -v "^# [A-Za-z:& ]*: " gpurun_out/${TAG}_sedov400.log
timeout -k 10 240 python -u bench.py --init evrard -n 200 --steps 10 --warmup 3 --verbose > gpurun_out/${TAG}_evrard200.log 2>&1 || { tail -20 gpurun_out/${TAG}_evrard200.log; exit 1; }
grep -v "^# [A-Za-z:& ]*: " gpurun_out/${TAG}_evrard200.log
