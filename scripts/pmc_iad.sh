#!/bin/bash
# counter passes for the IAD kernel (Sedov -n 200): issue/wait breakdown and texture/L1 pipeline utilisation
set -o pipefail
OUT=gpurun_out/pmc_iad; mkdir -p $OUT; export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
B="python3 bench.py -n 200 --steps 1 --warmup 1"
RX="iadDivvCurlv|momentumEnergyVe"
timeout -s KILL 120 rocprofv3 --kernel-include-regex "$RX" --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM --output-format csv -d $OUT/p1 -o run -- $B > $OUT/p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-include-regex "$RX" --pmc TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE --output-format csv -d $OUT/p2 -o run -- $B > $OUT/p2.log 2>&1
echo "exit $?"
