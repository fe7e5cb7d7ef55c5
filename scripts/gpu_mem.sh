#!/bin/bash
# memory: per-substep device-memory peaks (SPHX_MEM_TRACE) and the between-steps census, Sedov -n 200
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/mem; mkdir -p $O; export TMPDIR=/tmp
SPHX_MEM_TRACE=1 timeout -k 10 300 python3 bench.py --init sedov -n ${N:-200} --steps 2 --warmup 1 --verbose > $O/trace.out 2> $O/trace.err || { tail -5 $O/trace.err; exit 1; }
grep "memory peak\|peak_mem" $O/trace.err $O/trace.out | head -30
timeout -k 10 300 python3 scripts/mem_census.py --init sedov -n ${N:-200} --steps 2 > $O/census.txt 2>&1 || { tail -5 $O/census.txt; exit 1; }
cat $O/census.txt | tail -30
