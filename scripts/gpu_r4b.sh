#!/bin/bash
# A/B of the 2-rank-one-GPU VE step test: previous round's tree (_old) vs the current one
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/r4b; mkdir -p $O; export TMPDIR=/tmp
(cd _old && timeout -k 10 200 python3 -u -m pytest tests/test_distributed_gpu.py -m gpu -x -q -k ve_step --timeout 150 --timeout-method thread > $O/old.log 2>&1); echo "old rc $?"; tail -3 $O/old.log
timeout -k 10 200 python3 -u -m pytest tests/test_distributed_gpu.py -m gpu -x -q -k ve_step --timeout 150 --timeout-method thread > $O/new.log 2>&1; echo "new rc $?"; tail -3 $O/new.log
timeout -k 10 200 python3 -u scripts/diag_2rank.py > $O/diag.log 2>&1; echo "diag rc $?"; tail -20 $O/diag.log
bash scripts/gpu_r4a.sh
