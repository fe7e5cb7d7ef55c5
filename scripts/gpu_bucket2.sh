#!/bin/bash
# leaf capacity 256 vs 128 on Noh -n 300 and Sedov -n 400 (headline), 64 vs 128 on Sedov -n 400
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/bucket2; mkdir -p $O; export TMPDIR=/tmp
for c in "noh 300 256" "noh 300 128" "sedov 400 128" "sedov 400 256" "sedov 400 64" "sedov 400 128"; do
  set -- $c
  SPHX_BUCKET_FOCUS=$3 timeout -k 10 400 python3 bench.py --init $1 -n $2 --steps 5 --warmup 3 > $O/$1_$3.json 2> $O/$1_$3.err || { echo "$c failed"; tail -5 $O/$1_$3.err; exit 1; }
  echo "$c: $(grep -o '"ms_per_step": [0-9.]*\|"peak_mem_gib": [0-9.]*' $O/$1_$3.json | tr '\n' ' ')"
done
