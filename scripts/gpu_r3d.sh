#!/bin/bash
# round-3 session-3 measurements: gravity leaf-size what-if, then the per-GPU shares of the 8-GPU Noh / Turbulence
# configs with kernel statistics (search share after the round-3 search rewrite)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r3d; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 240 python3 -u scripts/grav_bucket.py -n 200 > $OUT/grav_bucket.log 2>&1 || { tail -20 $OUT/grav_bucket.log; exit 1; }
cat $OUT/grav_bucket.log
for c in "noh 300 ve" "turbulence 600 turbulence"; do
  set -- $c
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$1 -o run -- \
      python3 bench.py --init $1 -n $2 --prop $3 --steps 3 --warmup 1 > $OUT/$1.log 2>&1 || { tail -20 $OUT/$1.log; exit 1; }
  grep -E '^\{' $OUT/$1.log
  python3 scripts/kernel_table.py $OUT/$1/run_kernel_stats.csv 4 > $OUT/$1_kernels.md
  head -8 $OUT/$1_kernels.md
done
