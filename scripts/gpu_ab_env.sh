#!/bin/bash
# A/B of environment settings on one bench config: bash scripts/gpu_ab_env.sh "ARGS" TAG1 "ENV1" TAG2 "ENV2" ...
# (ENV: space-separated VAR=VALUE assignments, "-" for none). Substep summary lines only.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
ARGS=$1; shift
while [ $# -ge 2 ]; do
    tag=$1; envs=$2; shift 2
    [ "$envs" = "-" ] && envs=""
    env $envs timeout -k 10 240 python -u bench.py $ARGS --verbose > gpurun_out/ab/$tag.log 2>&1 || { echo "$tag failed"; tail -20 gpurun_out/ab/$tag.log; exit 1; }
    echo "== $tag ($envs)"; grep -E '"ms_per_step"|^# substep|^# max mem' gpurun_out/ab/$tag.log | sed -e 's/.*"ms_per_step": \([0-9.]*\).*/ms_per_step \1/'
done
