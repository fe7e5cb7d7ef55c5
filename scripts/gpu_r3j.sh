#!/bin/bash
# reduction/time-step kernel tests + case tests, default bench, GPU-busy at the 8-GPU per-rank shares
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_reduce.py tests/test_octree.py tests/test_gravity.py tests/test_gpu_cases.py tests/test_syncs_gpu.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/r3j_tests.log 2>&1 || { tail -30 gpurun_out/r3j_tests.log; exit 1; }
tail -2 gpurun_out/r3j_tests.log
timeout -k 10 400 python3 bench.py > gpurun_out/r3j_bench.json 2> gpurun_out/r3j_bench.err || { tail -20 gpurun_out/r3j_bench.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"evrard_ms_per_step": [0-9.]*' gpurun_out/r3j_bench.json
bash scripts/profile_busy.sh r3j_evrard100 --init evrard -n 100 | head -1
bash scripts/profile_busy.sh r3j_sedov100 --init sedov -n 100 | head -1
