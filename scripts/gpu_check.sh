#!/bin/bash
# GPU tests + short Sedov/Evrard benches (used after each change that touches the GPU path)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-check}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s ${PYTEST_SEL} --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gputests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/${TAG}_gputests.log; exit 1; }
tail -3 gpurun_out/${TAG}_gputests.log
grep "fixed-point vs fp64" gpurun_out/${TAG}_gputests.log
timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 > gpurun_out/${TAG}_sedov.log 2>&1 || { tail -20 gpurun_out/${TAG}_sedov.log; exit 1; }
grep metric gpurun_out/${TAG}_sedov.log | cut -c1-400
timeout -k 10 240 python -u bench.py --init evrard -n 200 --steps 10 --warmup 3 --verbose > gpurun_out/${TAG}_evrard.log 2>&1 || { tail -20 gpurun_out/${TAG}_evrard.log; exit 1; }
grep "metric\|substep\|stats" gpurun_out/${TAG}_evrard.log | cut -c1-400
