#!/bin/bash
# counter passes for the neighbor search kernel (Sedov -n 200)
set -o pipefail
OUT=gpurun_out/pmc_search; mkdir -p $OUT; export TMPDIR=/tmp
B="python3 bench.py -n 200 --steps 1 --warmup 1"
RX="findNeighborsKernel|iadDivvCurlv"
timeout -s KILL 120 rocprofv3 --kernel-include-regex "$RX" --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU --output-format csv -d $OUT/p1 -o run -- $B > $OUT/p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-include-regex "$RX" --pmc TA_TA_BUSY_sum TA_FLAT_WRITE_WAVEFRONTS_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE --output-format csv -d $OUT/p2 -o run -- $B > $OUT/p2.log 2>&1
echo "exit $?"
