#!/bin/bash
# box prefetch: GPU tests of the step, Evrard -n 100 bench + busy, Evrard -n 200 busy
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/boxpf; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_cases.py tests/test_syncs_gpu.py tests/test_gpu_parity.py tests/test_gravity.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 1 2; do
  timeout -k 10 200 python3 bench.py --init evrard -n 100 --steps 30 --warmup 5 > $O/e100_$k.json 2> $O/e100_$k.err || { tail -5 $O/e100_$k.err; exit 1; }
  echo "e100 bench $k: $(grep -o '"ms_per_step": [0-9.]*' $O/e100_$k.json)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pe100 -o run -- \
    python3 bench.py --init evrard -n 100 --steps 8 --warmup 3 > $O/pe100.log 2>&1 || { tail -5 $O/pe100.log; exit 1; }
python3 scripts/gpu_busy.py $O/pe100/run_kernel_trace.csv 8 > $O/e100_busy.txt; head -1 $O/e100_busy.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pe200 -o run -- \
    python3 bench.py --init evrard -n 200 --steps 6 --warmup 4 > $O/pe200.log 2>&1 || { tail -5 $O/pe200.log; exit 1; }
python3 scripts/gpu_busy.py $O/pe200/run_kernel_trace.csv 6 > $O/e200_busy.txt; head -1 $O/e200_busy.txt
