#!/bin/bash
# A/B of HIP tuning variants (built locally with `python -m sphexa_amd.build_native --variant TAG -D...`):
# one short bench per variant, default build first. usage: bash scripts/sweep_variants.sh N TAG...
set -o pipefail
N=${1:-200}
shift
mkdir -p gpurun_out/sweep
timeout -k 10 300 python bench.py -n "$N" --steps 3 --warmup 1 --verbose > gpurun_out/sweep/default.log 2>&1 || exit $?
for tag in "$@"; do
    SPHX_HIP_VARIANT=$tag timeout -k 10 300 python bench.py -n "$N" --steps 3 --warmup 1 --verbose \
        > gpurun_out/sweep/$tag.log 2>&1 || exit $?
done
