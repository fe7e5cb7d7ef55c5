#!/bin/bash
# gravity development pass: GPU gravity tests (+ spill/fallback paths), accuracy A/B, Evrard -n 200 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gravity.py tests/test_gpu_parity.py -k "gravity" -m gpu -x -v \
    --timeout 120 --timeout-method thread > gpurun_out/grav_tests.log 2>&1 || { tail -40 gpurun_out/grav_tests.log; exit 1; }
tail -2 gpurun_out/grav_tests.log
bash scripts/gpu_grav_ab.sh "$@"
