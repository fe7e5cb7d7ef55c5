#!/bin/bash
# end-of-session validation: full GPU test suite, default bench, kernel tables of both headline configs
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3f_tests.log 2>&1 \
    || { tail -30 gpurun_out/r3f_tests.log; exit 1; }
tail -1 gpurun_out/r3f_tests.log
timeout -k 10 400 python3 bench.py > gpurun_out/r3f_bench.json 2> gpurun_out/r3f_bench.err || { tail -20 gpurun_out/r3f_bench.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"evrard_ms_per_step": [0-9.]*' gpurun_out/r3f_bench.json
bash scripts/prof_cases.sh r3fprof > gpurun_out/r3fprof.txt 2>&1 || { tail -20 gpurun_out/r3fprof.txt; exit 1; }
head -8 gpurun_out/r3fprof.txt
