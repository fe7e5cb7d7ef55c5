#!/bin/bash
# neighbor-search statistics on glass and lattice ICs (rounds, touched leaves, staged candidates, hits, paths) and the
# micro-benchmarks mirroring the reference's hilbert.cu / octree.cu / neighbor_driver.cu
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/sstats; mkdir -p $O; export TMPDIR=/tmp
export SPHX_SEARCH_STATS=1
for c in "sedov -n 200" "noh -n 300" "evrard -n 100" "evrard -n 200" "turbulence -n 200"; do
  set -- $c
  timeout -k 10 300 python3 bench.py --init $1 -n $3 --steps 2 --warmup 1 --verbose > $O/$1$3.out 2> $O/$1$3.err || { echo "$c failed"; tail -5 $O/$1$3.err; exit 1; }
  echo "== $c"; grep "neighbor search\|substep FindNeighbors" $O/$1$3.err
done
unset SPHX_SEARCH_STATS
timeout -k 10 300 python3 scripts/micro_bench.py > $O/micro.txt 2>&1 || { tail -5 $O/micro.txt; exit 1; }
cat $O/micro.txt
