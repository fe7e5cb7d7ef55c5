#!/bin/bash
# selected GPU tests (first argument, quoted), then the default bench. usage: bash scripts/gpu_seq.sh TAG "tests/x.py tests/y.py"
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1; T=${2:-tests}
timeout -k 10 500 python -u -m pytest $T -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
[ "$3" = nobench ] && exit 0
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --verbose > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
grep -E "case|substep (domain|Find|Mom|Grav)" gpurun_out/${TAG}_bench.log
