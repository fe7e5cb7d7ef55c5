#!/bin/bash
# neighbor-search path statistics of the benchmark cases (verbose bench, 2 steps each)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/paths; mkdir -p $O; export TMPDIR=/tmp
for c in "sedov -n 200" "noh -n 300" "evrard -n 100" "evrard -n 200" "turbulence -n 200"; do
  set -- $c
  timeout -k 10 300 python3 bench.py --init $1 -n $3 --steps 2 --warmup 1 --verbose > $O/$1$3.out 2> $O/$1$3.err || { echo "$c failed"; tail -5 $O/$1$3.err; exit 1; }
  echo "== $c"; grep "neighbor search" $O/$1$3.err
done
