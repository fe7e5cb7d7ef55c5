#!/bin/bash
# same-box anchor: the reference (sekelle/SPH-EXA, hipified + built here for gfx950, binary in _refbuild/) on the
# headline configs, then ours. Outputs under gpurun_out/ref/.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/ref; mkdir -p $O; cd $O
export LD_LIBRARY_PATH=/usr/lib/x86_64-linux-gnu  # the binary's runpath puts conda's older libstdc++ first
export OMP_NUM_THREADS=16
timeout -k 10 400 $R/_refbuild/sphexa-hip --init sedov -n ${SN:-400} -s ${STEPS:-12} > sedov.log 2>&1
echo "sedov rc $?"; grep -E "Total time for iteration|Total execution time" sedov.log | tail -4
timeout -k 10 400 $R/_refbuild/sphexa-hip --init evrard -n ${EN:-200} -s ${STEPS:-12} --glass $R/_refbuild/glass16.h5 > evrard.log 2>&1
echo "evrard rc $?"; grep -E "Total time for iteration|Total execution time|Total Neighbors|Particles:" evrard.log | tail -5
cd $R
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 > $O/ours.json 2> $O/ours.err || { tail -5 $O/ours.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"evrard_ms_per_step": [0-9.]*' $O/ours.json
