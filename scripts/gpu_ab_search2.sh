#!/bin/bash
# search A/B on three cases (search_timing.py), default vs the variants given; then the search parity tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/abs; mkdir -p $OUT; export TMPDIR=/tmp
for c in "sedov 400" "noh 300" "evrard 200"; do
  set -- $c
  for v in default "${VARIANTS[@]}" $EXTRA; do
    if [ $v = default ]; then unset SPHX_HIP_VARIANT; else export SPHX_HIP_VARIANT=$v; fi
    timeout -k 10 240 python -u scripts/search_timing.py --init $1 -n $2 --reps 5 > $OUT/$1$2_$v.log 2>&1 || { tail -20 $OUT/$1$2_$v.log; exit 1; }
    echo "$1 $2 $v: $(grep search $OUT/$1$2_$v.log | tail -1)"
  done
done
unset SPHX_HIP_VARIANT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "neighbor or spill or subgroup or chunk" \
    --timeout 150 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log; exit $rc
