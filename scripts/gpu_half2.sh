#!/bin/bash
# half-box gravity lists: micro-benchmark with statistics, spill/chunk tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/half2; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 200 python3 scripts/grav_micro.py -n 200 -k 3 > $O/micro.log 2>&1; rc=$?; tail -4 $O/micro.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread \
    -k "spill or chunk or subgroup" > $O/tests.log 2>&1; rc=$?; tail -15 $O/tests.log; exit $rc
