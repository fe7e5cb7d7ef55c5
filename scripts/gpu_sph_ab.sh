#!/bin/bash
# SPH timing A/B of HIP build variants on Sedov (default -n 200; N=... to change), 3 timed steps, substeps printed
set -o pipefail
mkdir -p gpurun_out/ab
N=${N:-200}
for tag in default "$@"; do
    if [ "$tag" = default ]; then unset SPHX_HIP_VARIANT; else export SPHX_HIP_VARIANT=$tag; fi
    log=gpurun_out/ab/${tag}_sedov$N.log
    timeout -k 10 300 python bench.py -n $N --steps ${STEPS:-3} --warmup ${WARMUP:-2} --verbose > $log 2>&1 || { tail -20 $log; exit 1; }
    echo "$tag: step $(grep -E '^\{' $log | python -c "import json,sys; print(round(json.loads(sys.stdin.read())['ms_per_step'],2))") ms |" \
        $(grep -E '^# substep' $log | awk '$NF=="ms/step" && $(NF-1)>0.3 {printf "%s=%s ", $3, $(NF-1)}')
done
