#!/bin/bash
# gravity A/B: accuracy vs direct sum and Evrard -n 200 timing for the default build and each variant given
set -o pipefail
mkdir -p gpurun_out/grav_ab
for tag in default "$@"; do
    if [ "$tag" = default ]; then unset SPHX_HIP_VARIANT; else export SPHX_HIP_VARIANT=$tag; fi
    timeout -k 10 120 python scripts/gravity_accuracy.py 20000 > gpurun_out/grav_ab/acc_$tag.log 2>&1 || { cat gpurun_out/grav_ab/acc_$tag.log; exit 1; }
    cat gpurun_out/grav_ab/acc_$tag.log | grep -v amdgpu.ids
    timeout -k 10 300 python bench.py --init evrard -n 200 --steps 3 --warmup 1 --verbose \
        > gpurun_out/grav_ab/bench_$tag.log 2>&1 || { tail -20 gpurun_out/grav_ab/bench_$tag.log; exit 1; }
    grep -E 'substep Gravity|gravity stats' gpurun_out/grav_ab/bench_$tag.log
    grep -E '^\{' gpurun_out/grav_ab/bench_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', 'ms/step', round(d['ms_per_step'],2), 'Mp-upd/s', round(d['value']/1e6,1))"
done
