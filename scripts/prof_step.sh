#!/bin/bash
# Kernel-trace statistics of a few Sedov -n 400 steps plus one SQ counter pass over the pair-loop kernels.
# usage: bash scripts/prof_step.sh TAG [variant]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; VAR=${2:-}
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
[ -n "$VAR" ] && export SPHX_HIP_VARIANT=$VAR
B="python3 bench.py --init sedov -n 400 --steps 2 --warmup 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- $B > $OUT/kt.log 2>&1 || { tail -5 $OUT/kt.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-include-regex "Kernel" --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/pmc -o run -- python3 bench.py --init sedov -n 400 --steps 1 --warmup 0 > $OUT/pmc.log 2>&1 || { tail -5 $OUT/pmc.log; exit 1; }
echo prof done
