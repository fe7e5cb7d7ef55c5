#!/bin/bash
# steady-state per-GPU shares of the 8-GPU Noh / Turbulence configs (enough warmup for the allocator to settle)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r3cases; mkdir -p $OUT
timeout -k 10 300 python3 bench.py --init noh -n 300 --steps 5 --warmup 3 > $OUT/noh.json 2> $OUT/noh.err || { tail -5 $OUT/noh.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $OUT/noh.json
timeout -k 10 600 python3 bench.py --init turbulence -n 600 --prop turbulence --steps 3 --warmup 3 > $OUT/turb.json 2> $OUT/turb.err || { tail -5 $OUT/turb.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"peak_mem_gib": [0-9.]*' $OUT/turb.json
