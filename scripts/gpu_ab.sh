#!/bin/bash
# timing A/B of HIP build variants on Evrard -n 200 (gravity + SPH) and Sedov -n 200 (SPH):
# usage: bash scripts/gpu_ab.sh VARIANT...   (default build always first)
set -o pipefail
mkdir -p gpurun_out/ab
for tag in default "$@"; do
    if [ "$tag" = default ]; then unset SPHX_HIP_VARIANT; else export SPHX_HIP_VARIANT=$tag; fi
    for cfg in "evrard 200" "sedov 200"; do
        set -- $cfg
        log=gpurun_out/ab/${tag}_$1.log
        timeout -k 10 300 python bench.py --init $1 -n $2 --steps 3 --warmup 2 --verbose > $log 2>&1 || { tail -20 $log; exit 1; }
        echo "$tag $1: step $(grep -E '^\{' $log | python -c "import json,sys; print(round(json.loads(sys.stdin.read())['ms_per_step'],2))") ms |" \
            $(grep -E '^# substep' $log | awk '$NF=="ms/step" && $(NF-1)>0.3 {printf "%s=%s ", $3, $(NF-1)}')
    done
done
