#!/bin/bash
# gravity A/B (cost order, MFMA pipelining) + Noh -n 300 search spill check
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_grav_order.sh go2 nopipe m2ppipe m2porder || exit 1
OUT=gpurun_out/r3f; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/noh -o run -- \
    python3 bench.py --init noh -n 300 --steps 3 --warmup 2 > $OUT/noh.log 2>&1 || { tail -20 $OUT/noh.log; exit 1; }
grep -E '^\{' $OUT/noh.log | cut -c1-200
python3 scripts/kernel_table.py $OUT/noh/run_kernel_stats.csv 5 10 > $OUT/noh_kernels.md; cat $OUT/noh_kernels.md
