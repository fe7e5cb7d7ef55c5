#!/bin/bash
# Neighbor-search A/B and counters on one MI355X (Sedov -n 400 initial conditions):
#   search alone, this build vs an optional variant (SPHX_HIP_VARIANT), then kernel trace + one SQ counter pass of
#   findNeighborsKernel. usage: bash scripts/prof_search.sh TAG [variant]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-search}; VAR=${2:-}
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/search_timing.py --init sedov -n 400 --reps 5 > $OUT/time_new.log 2>&1 || { tail -20 $OUT/time_new.log; exit 1; }
cat $OUT/time_new.log | grep search
if [ -n "$VAR" ]; then
  SPHX_HIP_VARIANT=$VAR timeout -k 10 200 python -u scripts/search_timing.py --init sedov -n 400 --reps 5 > $OUT/time_$VAR.log 2>&1 || { tail -20 $OUT/time_$VAR.log; exit 1; }
  cat $OUT/time_$VAR.log | grep search
fi
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 scripts/search_timing.py --init sedov -n 400 --reps 3 > $OUT/kt.log 2>&1 || { tail -20 $OUT/kt.log; exit 1; }
timeout -s KILL 200 rocprofv3 --kernel-include-regex "findNeighborsKernel" --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/pmc -o run -- python3 scripts/search_timing.py --init sedov -n 400 --reps 2 > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
echo done
