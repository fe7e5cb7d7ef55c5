#!/bin/bash
# full GPU suite + smoke, Evrard/Sedov -n 100 busy, Sedov -n 400 steady-state kernels, default bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/r4z; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -10 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for c in "evrard 100" "sedov 100"; do
  set -- $c
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$1 -o run -- \
      python3 bench.py --init $1 -n $2 --steps 8 --warmup 3 > $O/p$1.log 2>&1 || { tail -5 $O/p$1.log; exit 1; }
  python3 scripts/gpu_busy.py $O/p$1/run_kernel_trace.csv 8 > $O/$1$2_busy.txt; echo "$c: $(head -1 $O/$1$2_busy.txt)"
done
for k in 1 2; do
  timeout -k 10 200 python3 bench.py --init evrard -n 100 --steps 30 --warmup 5 > $O/e100_$k.json 2> $O/e100_$k.err || { tail -5 $O/e100_$k.err; exit 1; }
  echo "e100 bench $k: $(grep -o '"ms_per_step": [0-9.]*' $O/e100_$k.json)"
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ps400 -o run -- \
    python3 bench.py --init sedov -n 400 --steps 4 --warmup 3 > $O/s400.json 2> $O/s400.err || { tail -5 $O/s400.err; exit 1; }
python3 scripts/gpu_busy.py $O/ps400/run_kernel_trace.csv 4 > $O/s400_busy.txt; head -1 $O/s400_busy.txt
rm -f $O/ps400/run_kernel_trace.csv
timeout -k 10 400 python3 bench.py --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"evrard_ms_per_step": [0-9.]*\|"peak_mem_gib": [0-9.]*' $O/bench.json | tr '\n' ' '
