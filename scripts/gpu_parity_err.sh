#!/bin/bash
# GPU-vs-OpenMP errors of the step parity tests (printed), to size their tolerances
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/parity; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cases.py -m gpu -x -q -s --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
grep -h "GPU vs OpenMP\|^noh\|^evrard\|^isobaric\|^gresho\|^wind\|^kelvin" $O/tests.log
