#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/mem; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/mem_census.py --init sedov -n ${N:-200} --steps 3 --at-sync > $O/census_sync.txt 2>&1 || { tail -5 $O/census_sync.txt; exit 1; }
grep -v "Warning\|reduce_op\|amdgpu" $O/census_sync.txt
