#!/bin/bash
# Kernel-trace statistics of the two headline configs (Sedov -n 400: 2 steps, Evrard -n 200: 3 steps) and a table of the
# top kernels per case. usage: bash scripts/prof_cases.sh TAG [variant]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; VAR=${2:-}
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
[ -n "$VAR" ] && export SPHX_HIP_VARIANT=$VAR
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/sedov -o run -- \
    python3 bench.py --init sedov -n 400 --steps 2 --warmup 1 > $OUT/sedov.log 2>&1 || { tail -5 $OUT/sedov.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/evrard -o run -- \
    python3 bench.py --init evrard -n 200 --steps 3 --warmup 2 > $OUT/evrard.log 2>&1 || { tail -5 $OUT/evrard.log; exit 1; }
for c in sedov evrard; do
  echo "== $c"; python3 scripts/kernel_table.py $OUT/$c/run_kernel_stats.csv $([ $c = sedov ] && echo 3 || echo 5)
done
