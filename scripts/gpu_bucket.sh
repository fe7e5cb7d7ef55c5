#!/bin/bash
# local octree leaf capacity (bucketSizeFocus) A/B: Noh -n 300 (glass), Sedov -n 200 (lattice), Evrard -n 100
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/bucket; mkdir -p $O; export TMPDIR=/tmp
for c in "noh 300" "sedov 200" "evrard 100" "turbulence 200"; do
  set -- $c
  for b in 64 32 128 64; do
    SPHX_BUCKET_FOCUS=$b timeout -k 10 300 python3 bench.py --init $1 -n $2 --steps 6 --warmup 3 > $O/$1_$b.json 2> $O/$1_$b.err || { echo "$c $b failed"; tail -5 $O/$1_$b.err; exit 1; }
    echo "$c bucket $b: $(grep -o '"ms_per_step": [0-9.]*' $O/$1_$b.json)"
  done
done
