#!/bin/bash
# SQ counter passes of the search kernel (Sedov -n 400 ICs, search alone), for this build and optional variants.
# usage: bash scripts/pmc_search2.sh TAG [variant ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; shift
export TMPDIR=/tmp
B="python3 scripts/search_timing.py --init sedov -n 400 --reps 2"
for v in default "$@"; do
  OUT=gpurun_out/$TAG/$v; mkdir -p $OUT
  if [ "$v" != default ]; then export SPHX_HIP_VARIANT=$v; else unset SPHX_HIP_VARIANT; fi
  timeout -s KILL 200 rocprofv3 --kernel-include-regex "findNeighborsKernel" --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/p1 -o run -- $B > $OUT/p1.log 2>&1 || exit 1
  timeout -s KILL 200 rocprofv3 --kernel-include-regex "findNeighborsKernel" --pmc SQ_WAVES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/p2 -o run -- $B > $OUT/p2.log 2>&1 || exit 1
  echo "pmc $v done"
done
