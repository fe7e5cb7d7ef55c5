#!/bin/bash
# LDS A/B: bank-conflict counters of the cooperative-gather SPH loops for the default build and the variants given
# as arguments, then substep timings (Sedov -n $N). usage: bash scripts/ab_lds.sh [variant...]
set -o pipefail
mkdir -p gpurun_out
for v in default "$@"; do
  if [ $v = default ]; then unset SPHX_HIP_VARIANT; else export SPHX_HIP_VARIANT=$v; fi
  OUT=gpurun_out/lds_$v; mkdir -p $OUT
  timeout -s KILL 200 rocprofv3 --kernel-include-regex "iadDivv|momentumEnergyVe|avSwitches" --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $OUT -o run -- python3 bench.py -n ${N:-200} --steps 1 --warmup 1 > $OUT/log 2>&1 || exit 1
done
N=${N:-200} STEPS=3 WARMUP=2 bash scripts/gpu_sph_ab.sh "$@"
