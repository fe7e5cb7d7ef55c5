#!/bin/bash
# host synchronizations per step: 1 rank (Evrard, Sedov) and 2 ranks sharing the GPU over gloo (staging excluded)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-syncs}
timeout -k 10 200 python -u scripts/sync_inventory.py --init evrard -n 50 > gpurun_out/${TAG}_evrard1.txt 2>&1 || { tail -20 gpurun_out/${TAG}_evrard1.txt; exit 1; }
timeout -k 10 200 python -u scripts/sync_inventory.py --init sedov -n 50 > gpurun_out/${TAG}_sedov1.txt 2>&1 || { tail -20 gpurun_out/${TAG}_sedov1.txt; exit 1; }
timeout -k 10 300 python -u scripts/sync_inventory.py --ranks 2 --init evrard -n 50 > gpurun_out/${TAG}_evrard2.txt 2>&1 || { tail -20 gpurun_out/${TAG}_evrard2.txt; exit 1; }
timeout -k 10 300 python -u scripts/sync_inventory.py --ranks 2 --init sedov -n 50 > gpurun_out/${TAG}_sedov2.txt 2>&1 || { tail -20 gpurun_out/${TAG}_sedov2.txt; exit 1; }
grep -h -A30 "synchronizing" gpurun_out/${TAG}_*.txt
