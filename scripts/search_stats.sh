#!/bin/bash
# search statistics (staged candidates, hits, sub-group what-if) on Sedov -n 400 and Evrard -n 200 ICs with the
# 'stats' build variant (SPHX_NS_STATS). usage: bash scripts/search_stats.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$1; mkdir -p $OUT
SPHX_SEARCH_STATS=1 SPHX_HIP_VARIANT=stats timeout -k 10 200 python -u scripts/search_timing.py --init sedov -n 400 --reps 2 > $OUT/sedov.log 2>&1 || { tail $OUT/sedov.log; exit 1; }
grep "search\|per group" $OUT/sedov.log
SPHX_SEARCH_STATS=1 SPHX_HIP_VARIANT=stats timeout -k 10 200 python -u scripts/search_timing.py --init evrard -n 200 --reps 2 > $OUT/evrard.log 2>&1 || { tail $OUT/evrard.log; exit 1; }
grep "search\|per group" $OUT/evrard.log
