#!/bin/bash
# leaf capacity with self-gravity on one rank: Evrard -n 200 at 64 / 128 / 256
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/bucket5; mkdir -p $O; export TMPDIR=/tmp
for b in 64 128 256 64 128 256; do
  SPHX_BUCKET_FOCUS=$b timeout -k 10 400 python3 bench.py --init evrard -n 200 --steps 6 --warmup 3 > $O/e200_$b.json 2> $O/e200_$b.err || { echo "$b failed"; tail -5 $O/e200_$b.err; exit 1; }
  echo "evrard 200 bucket $b: $(grep -o '"ms_per_step": [0-9.]*' $O/e200_$b.json)"
done
