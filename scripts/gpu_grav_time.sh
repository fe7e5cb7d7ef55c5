#!/bin/bash
# gravity timing A/B only (Evrard -n 200, 3 timed steps after 2 warmup): default build + variants given
set -o pipefail
mkdir -p gpurun_out/grav_ab
for tag in default "$@"; do
    if [ "$tag" = default ]; then unset SPHX_HIP_VARIANT; else export SPHX_HIP_VARIANT=$tag; fi
    timeout -k 10 300 python bench.py --init evrard -n 200 --steps 3 --warmup 2 --verbose \
        > gpurun_out/grav_ab/bench_$tag.log 2>&1 || { tail -20 gpurun_out/grav_ab/bench_$tag.log; exit 1; }
    echo "$tag: $(grep -E '^# Gravity' gpurun_out/grav_ab/bench_$tag.log | tail -3 | awk '{printf "%.1f ", $3*1000}') ms" \
         "| step $(grep -E '^\{' gpurun_out/grav_ab/bench_$tag.log | python -c "import json,sys; print(round(json.loads(sys.stdin.read())['ms_per_step'],2))")"
done
