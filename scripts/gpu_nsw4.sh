#!/bin/bash
# neighbor-search occupancy A/B at the new leaf capacities: 5 (default) vs 4 waves per SIMD
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/nsw4; mkdir -p $O; export TMPDIR=/tmp
for c in "sedov 200" "noh 300" "sedov 400"; do
  set -- $c
  for v in default nsw4 default nsw4; do
    if [ $v = default ]; then unset SPHX_HIP_VARIANT; else export SPHX_HIP_VARIANT=$v; fi
    timeout -k 10 400 python3 bench.py --init $1 -n $2 --steps 5 --warmup 3 > $O/$1$2_$v.json 2> $O/$1$2_$v.err || { echo "$c $v failed"; tail -5 $O/$1$2_$v.err; exit 1; }
    echo "$c $v: $(grep -o '"ms_per_step": [0-9.]*' $O/$1$2_$v.json)"
  done
done
