#!/bin/bash
# speculative XMass -> Gradh -> EOS chain: GPU tests of the VE step, Evrard -n 100 / Sedov -n 100 busy, default bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/chain; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_cases.py tests/test_syncs_gpu.py tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 1 2; do
  timeout -k 10 200 python3 bench.py --init evrard -n 100 --steps 30 --warmup 5 > $O/e100_$k.json 2> $O/e100_$k.err || { tail -5 $O/e100_$k.err; exit 1; }
  echo "e100 bench $k: $(grep -o '"ms_per_step": [0-9.]*' $O/e100_$k.json)"
done
for c in "evrard 100" "sedov 100"; do
  set -- $c
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$1 -o run -- \
      python3 bench.py --init $1 -n $2 --steps 8 --warmup 3 > $O/p$1.log 2>&1 || { tail -5 $O/p$1.log; exit 1; }
  python3 scripts/gpu_busy.py $O/p$1/run_kernel_trace.csv 8 > $O/$1$2_busy.txt; echo "$c: $(head -1 $O/$1$2_busy.txt)"
done
timeout -k 10 400 python3 bench.py --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"evrard_ms_per_step": [0-9.]*\|"peak_mem_gib": [0-9.]*' $O/bench.json | tr '\n' ' '
