#!/bin/bash
# half-box gravity lists: gravity GPU tests, accuracy vs direct sum, per-kernel times on Evrard -n 200
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/half; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests/test_gravity.py tests/test_gravity_mpi.py tests/test_gpu_parity.py -m gpu -q \
    --timeout 150 --timeout-method thread -k "grav or Grav or spill or chunk or subgroup" > $O/tests.log 2>&1
rc=$?; tail -12 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 scripts/gravity_accuracy.py 50000 > $O/acc.log 2>&1 || { tail -20 $O/acc.log; exit 1; }
cat $O/acc.log
timeout -k 10 300 python3 scripts/debug_half2.py 100 200 > $O/nan.log 2>&1; rc=$?; cat $O/nan.log | grep "n="; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_grav_variants.sh "$@"
timeout -k 10 200 python3 scripts/grav_micro.py -n 200 -k 3 > $O/micro.log 2>&1; tail -3 $O/micro.log
