#!/bin/bash
# A/B of build variants on one Sedov bench each (10 steps). usage: bash scripts/ab_bench.sh TAG [init] v1 v2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; shift
INIT=sedov; N=400
if [ "$1" = evrard ]; then INIT=evrard; N=200; shift; fi
OUT=gpurun_out/$TAG; mkdir -p $OUT
for v in default "$@"; do
  if [ "$v" != default ]; then export SPHX_HIP_VARIANT=$v; else unset SPHX_HIP_VARIANT; fi
  timeout -k 10 300 python -u bench.py --init $INIT -n $N --steps 10 --warmup 3 --verbose > $OUT/$v.log 2>&1 || { tail -20 $OUT/$v.log; exit 1; }
  echo "$v: $(grep '# case' $OUT/$v.log)"
  grep "substep" $OUT/$v.log | grep -v "synchronizeHalos\|Equation\|Timestep"
done
