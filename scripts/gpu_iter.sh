#!/bin/bash
# Iteration pass on one MI355X: selected GPU tests, then the default bench (Sedov -n 400 + Evrard -n 200, --verbose substeps).
# usage: bash scripts/gpu_iter.sh TAG [pytest targets...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-iter}; shift
TESTS=${@:-tests}
timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
# default bench: Sedov -n 400 then Evrard -n 200 in one invocation (the driver's command)
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --verbose > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
grep -v "^# [A-Za-z:& ]*: " gpurun_out/${TAG}_bench.log
