#!/bin/bash
# leaf capacity 128 vs 256 across hydro cases and sizes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/bucket3; mkdir -p $O; export TMPDIR=/tmp
for c in "sedov 100" "sedov 200" "turbulence 200" "noh 150" "gresho-chan 100" "sedov 400"; do
  set -- $c
  for b in 128 256 128 256; do
    SPHX_BUCKET_FOCUS=$b timeout -k 10 400 python3 bench.py --init $1 -n $2 --steps 6 --warmup 3 > $O/$1$2_$b.json 2> $O/$1$2_$b.err || { echo "$c $b failed"; tail -5 $O/$1$2_$b.err; exit 1; }
    echo "$c bucket $b: $(grep -o '"ms_per_step": [0-9.]*' $O/$1$2_$b.json)"
  done
done
