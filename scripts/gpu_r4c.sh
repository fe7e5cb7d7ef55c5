#!/bin/bash
# round 4: GPU tests, then old (_old, round-3 tree) vs new kernel tables on the same box
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/r4c; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest ${TESTS:-tests} -m gpu -q --maxfail=15 --timeout 150 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests.log | tail -2; grep FAILED $O/tests.log | head -15
[ $rc -gt 1 ] && { echo "pytest rc $rc: stopping"; tail -30 $O/tests.log; exit 1; }
prof() { # tree tag args...
  local tree=$1 tag=$2; shift 2
  (cd $tree && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o run -- \
      python3 bench.py --steps 3 --warmup 2 --verbose "$@" > $O/$tag.log 2>&1) || { echo "$tag failed"; tail -5 $O/$tag.log; return 1; }
  python3 scripts/kernel_table.py $O/$tag/run_kernel_stats.csv 5 > $O/$tag.md
  echo "== $tag"; head -14 $O/$tag.md | tail -11; grep "neighbor search:" $O/$tag.log || true
}
prof _old e100_old --init evrard -n 100 && prof . e100_new --init evrard -n 100 && \
prof _old e200_old --init evrard -n 200 && prof . e200_new --init evrard -n 200 && \
prof . noh300_new --init noh -n 300 && prof _old noh300_old --init noh -n 300 || exit 1
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"evrard_ms_per_step": [0-9.]*' $O/bench.json
