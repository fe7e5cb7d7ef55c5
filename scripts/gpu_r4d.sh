#!/bin/bash
# round 4: GPU tests, default bench, kernel tables (Evrard -n 100/200, Noh -n 300), Evrard -n 100 busy + sequence
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r4d}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest ${TESTS:-tests} -m gpu -q --maxfail=15 --timeout 150 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests.log | tail -2; grep FAILED $O/tests.log | head -15
[ $rc -gt 1 ] && { echo "pytest rc $rc: stopping"; tail -30 $O/tests.log; exit 1; }
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"evrard_ms_per_step": [0-9.]*\|"peak_mem_gib": [0-9.]*' $O/bench.json
prof() { # tag args...
  local tag=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o run -- \
      python3 bench.py --steps ${PSTEPS:-3} --warmup 2 "$@" > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -5 $O/$tag.log; return 1; }
  python3 scripts/kernel_table.py $O/$tag/run_kernel_stats.csv ${PSTEPS:-3} > $O/$tag.md
  echo "== $tag"; head -16 $O/$tag.md | tail -13
}
PSTEPS=5 prof e100 --init evrard -n 100 || exit 1
python3 scripts/gpu_busy.py $O/e100/run_kernel_trace.csv 4 > $O/e100_busy.txt; head -1 $O/e100_busy.txt
python3 scripts/step_sequence.py $O/e100/run_kernel_trace.csv -2 > $O/e100_seq.txt; tail -12 $O/e100_seq.txt
prof e200 --init evrard -n 200 && prof noh300 --init noh -n 300 || exit 1
