#!/bin/bash
# A/B of the evaluation-kernel dispatch order (Evrard -n 200): cost order (default build) vs SFC order (variant
# sfcorder, -DSPHX_GRAV_SFC_ORDER); kernel statistics per variant, then the gravity GPU tests on the default build.
# usage: bash scripts/gpu_grav_order.sh [TAG] [more variants...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-go}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
for v in default sfcorder "$@"; do
  if [ "$v" = default ]; then unset SPHX_HIP_VARIANT; else export SPHX_HIP_VARIANT=$v; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v -o run -- \
      python3 bench.py --init evrard -n 200 --steps 3 --warmup 2 > $OUT/$v.log 2>&1 || { tail -20 $OUT/$v.log; exit 1; }
  echo "== $v: $(grep -E '^\{' $OUT/$v.log | python3 -c "import json,sys; print(round(json.loads(sys.stdin.read())['ms_per_step'],2))") ms/step"
  python3 scripts/kernel_table.py $OUT/$v/run_kernel_stats.csv 5 8 | grep -E "kernel time|gravity"
done
unset SPHX_HIP_VARIANT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gravity.py \
    tests/test_gravity_mpi.py tests/test_multipole.py tests/test_gpu_parity.py > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log; exit $rc
