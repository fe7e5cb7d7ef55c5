#!/bin/bash
# A/B of neighbor-search build variants (search alone on Sedov -n 400 ICs). usage: bash scripts/ab_search.sh TAG v1 v2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 200 python -u scripts/search_timing.py --init sedov -n 400 --reps 5 > $OUT/default.log 2>&1 || { tail -20 $OUT/default.log; exit 1; }
grep search $OUT/default.log
for v in "$@"; do
  SPHX_HIP_VARIANT=$v timeout -k 10 200 python -u scripts/search_timing.py --init sedov -n 400 --reps 5 > $OUT/$v.log 2>&1 || { tail -20 $OUT/$v.log; exit 1; }
  grep search $OUT/$v.log
done
