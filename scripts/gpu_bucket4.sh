#!/bin/bash
# leaf capacity 256 vs 512 (hydro)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/bucket4; mkdir -p $O; export TMPDIR=/tmp
for c in "sedov 400" "sedov 100" "noh 300" "turbulence 200" "sedov 200"; do
  set -- $c
  for b in 256 512 256 512; do
    SPHX_BUCKET_FOCUS=$b timeout -k 10 400 python3 bench.py --init $1 -n $2 --steps 6 --warmup 3 > $O/$1$2_$b.json 2> $O/$1$2_$b.err || { echo "$c $b failed"; tail -5 $O/$1$2_$b.err; exit 1; }
    echo "$c bucket $b: $(grep -o '"ms_per_step": [0-9.]*' $O/$1$2_$b.json)"
  done
done
