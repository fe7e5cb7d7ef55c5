#!/bin/bash
# multi-rank bench rehearsal on the one-GPU box: N ranks share cuda:0 over gloo (RCCL refuses a shared device)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/shared; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gravity.py tests/test_gpu_reduce.py tests/test_distributed_gpu.py tests/test_gpu_cases.py \
    tests/test_syncs_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
export SPHX_BENCH_SHARED_GPU=1
for c in "2 sedov 150" "2 evrard 100" "4 sedov 150" "4 evrard 100"; do
  set -- $c
  timeout -k 10 300 python3 bench.py --gpus $1 --init $2 -n $3 --steps 4 --warmup 2 > $O/r$1_$2.json 2> $O/r$1_$2.err || { echo "$c failed"; tail -15 $O/r$1_$2.err; exit 1; }
  echo "$c: $(grep -o '"ms_per_step": [0-9.]*\|"backend": "[a-z]*"\|"ranks": [0-9]*' $O/r$1_$2.json | tr '\n' ' ')"
done
unset SPHX_BENCH_SHARED_GPU
for c in "sedov 150" "evrard 100"; do
  set -- $c
  timeout -k 10 300 python3 bench.py --init $1 -n $2 --steps 4 --warmup 2 > $O/r1_$1.json 2> $O/r1_$1.err || { echo "$c failed"; tail -5 $O/r1_$1.err; exit 1; }
  echo "1 $c: $(grep -o '"ms_per_step": [0-9.]*' $O/r1_$1.json)"
done
