#!/bin/bash
# full GPU test suite, default bench, GPU-busy of the 8-GPU per-rank share (Evrard -n 100)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3i_tests.log 2>&1 \
    || { tail -30 gpurun_out/r3i_tests.log; exit 1; }
tail -2 gpurun_out/r3i_tests.log
timeout -k 10 400 python3 bench.py > gpurun_out/r3i_bench.json 2> gpurun_out/r3i_bench.err || { tail -20 gpurun_out/r3i_bench.err; exit 1; }
cat gpurun_out/r3i_bench.json | grep -o '"ms_per_step": [0-9.]*\|"evrard_ms_per_step": [0-9.]*'
bash scripts/profile_busy.sh r3i_evrard100 --init evrard -n 100 | head -2
bash scripts/profile_busy.sh r3i_sedov100 --init sedov -n 100 | head -2
