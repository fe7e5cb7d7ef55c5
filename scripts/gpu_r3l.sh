#!/bin/bash
# full GPU tests, Evrard pair-loop path check, default bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3l_tests.log 2>&1 \
    || { tail -30 gpurun_out/r3l_tests.log; exit 1; }
tail -1 gpurun_out/r3l_tests.log
timeout -k 10 300 python3 bench.py --init evrard -n 200 --steps 2 --warmup 1 --verbose > gpurun_out/r3l_evrard_v.log 2>&1 || { tail -20 gpurun_out/r3l_evrard_v.log; exit 1; }
grep -m3 "pair-loop coordinates\|# substep Momentum\|# substep Gravity" gpurun_out/r3l_evrard_v.log
timeout -k 10 400 python3 bench.py > gpurun_out/r3l_bench.json 2> gpurun_out/r3l_bench.err || { tail -20 gpurun_out/r3l_bench.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"evrard_ms_per_step": [0-9.]*' gpurun_out/r3l_bench.json
