#!/bin/bash
# Counter passes for ONE kernel (regex) of a bench configuration: kernel stats + per-pass PMC sets.
# usage: bash scripts/profile_kernel.sh TAG KERNEL_REGEX [bench args...]
# output: gpurun_out/kprof_TAG/{stats,pmcA,pmcB,pmcC}
set -o pipefail
TAG=$1; RX=$2; shift 2
R=$(pwd)
OUT=$R/gpurun_out/kprof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
B="$R/bench.py --steps 1 --warmup 1 $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- python3 $B \
    > "$OUT/stats.log" 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --kernel-include-regex "$RX" --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
    SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d "$OUT/pmcA" -o run -- \
    python3 $B > "$OUT/pmcA.log" 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --kernel-include-regex "$RX" --pmc SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD \
    SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT \
    --output-format csv -d "$OUT/pmcB" -o run -- python3 $B > "$OUT/pmcB.log" 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --kernel-include-regex "$RX" --pmc SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES \
    SQ_INSTS_MFMA SQ_ACTIVE_INST_MISC TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/pmcC" -o run -- \
    python3 $B > "$OUT/pmcC.log" 2>&1
echo "pmcC exit $?"
