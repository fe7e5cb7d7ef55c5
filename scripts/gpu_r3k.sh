#!/bin/bash
# default bench + GPU-busy at the 8-GPU per-rank shares (after the fused-upsweep A/B)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python3 bench.py > gpurun_out/r3k_bench.json 2> gpurun_out/r3k_bench.err || { tail -20 gpurun_out/r3k_bench.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"evrard_ms_per_step": [0-9.]*' gpurun_out/r3k_bench.json
bash scripts/profile_busy.sh r3k_evrard100 --init evrard -n 100 | head -1
bash scripts/profile_busy.sh r3k_sedov100 --init sedov -n 100 | head -1
