#!/bin/bash
# memory-lean VE chain vs the momentum hand-off: Sedov -n 400 bench (ms/step, peak) both ways, then the VE GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/memab; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --init sedov -n 400 --steps 8 --warmup 2 > $O/lean.json 2> $O/lean.err || { tail -5 $O/lean.err; exit 1; }
echo "lean: $(grep -o '"ms_per_step": [0-9.]*\|"peak_mem_gib": [0-9.]*' $O/lean.json | tr '\n' ' ')"
SPHX_MOM_HANDOFF=1 timeout -k 10 300 python3 bench.py --init sedov -n 400 --steps 8 --warmup 2 > $O/ho.json 2> $O/ho.err || { tail -5 $O/ho.err; exit 1; }
echo "handoff: $(grep -o '"ms_per_step": [0-9.]*\|"peak_mem_gib": [0-9.]*' $O/ho.json | tr '\n' ' ')"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_guards.py -m gpu -q \
    --timeout 150 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; exit $rc
