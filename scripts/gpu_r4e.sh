#!/bin/bash
# golden (tier 3) + gravity tile tests, then the no-sched-barrier gravity variant
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/r4e; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_golden.py tests/test_gravity.py -m gpu -q --timeout 150 \
    --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -15 $O/tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_grav_variants.sh "$@"
