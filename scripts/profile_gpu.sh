#!/bin/bash
# Profiling pass used with gpurun (one GPU): 1-GPU bench with substep timings, rocprofv3 kernel stats and two PMC
# passes (SQ issue/wait breakdown + L2 hit rate; fetched bytes). Results under gpurun_out/prof_<tag>/.
# usage: bash scripts/profile_gpu.sh [N=200] [extra bench args...]
set -o pipefail
N=${1:-200}
shift || true
R=$(pwd)
OUT=$R/gpurun_out/prof_n${N}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python bench.py -n "$N" --steps 3 --warmup 1 --verbose "$@" > "$OUT/bench.log" 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- \
    python3 "$R/bench.py" -n "$N" --steps 2 --warmup 1 "$@" > "$OUT/stats.log" 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/pmc1" -o run -- \
    python3 "$R/bench.py" -n "$N" --steps 1 --warmup 1 "$@" > "$OUT/pmc1.log" 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv \
    -d "$OUT/pmc2" -o run -- python3 "$R/bench.py" -n "$N" --steps 1 --warmup 1 "$@" > "$OUT/pmc2.log" 2>&1
