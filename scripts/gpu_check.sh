#!/bin/bash
# One gpurun pass: GPU tests, smoke, then the two headline benches (Sedov -n 400, Evrard -n 200) with substep
# timings. Every GPU step has its own time limit; the chain stops at the first failure.
# usage: bash scripts/gpu_check.sh [tests|bench|all]
set -o pipefail
mkdir -p gpurun_out
what=${1:-all}
if [ "$what" = tests ] || [ "$what" = all ]; then
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
    tail -3 gpurun_out/gpu_tests.log
    timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
fi
if [ "$what" = bench ] || [ "$what" = all ]; then
    timeout -k 10 300 python bench.py --steps 5 --warmup 2 --verbose > gpurun_out/bench_sedov400.log 2>&1 || exit 1
    head -1 gpurun_out/bench_sedov400.log
    timeout -k 10 300 python bench.py --init evrard -n 200 --steps 5 --warmup 2 --verbose \
        > gpurun_out/bench_evrard200.log 2>&1 || exit 1
    head -1 gpurun_out/bench_evrard200.log
fi
