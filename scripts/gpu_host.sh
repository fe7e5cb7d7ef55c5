#!/bin/bash
# host-side profile of the Evrard -n 100 step (own time, then inclusive time of the domain/octree/search functions)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/host; mkdir -p $O
timeout -k 10 200 python3 scripts/host_profile.py --init evrard -n 100 --steps 20 --top 50 > $O/own.txt 2>&1 || { tail -5 $O/own.txt; exit 1; }
timeout -k 10 200 python3 scripts/host_profile.py --init evrard -n 100 --steps 20 --sort cumulative --top 80 \
    --filter 'sphexa_amd' > $O/cum.txt 2>&1 || { tail -5 $O/cum.txt; exit 1; }
head -3 $O/own.txt
