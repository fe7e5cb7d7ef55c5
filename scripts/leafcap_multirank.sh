#!/bin/bash
# Leaf capacity (bucketSizeFocus) of several ranks sharing one GPU over gloo on the glass hydro cases (verdict r5
# item 3): bench.py per (case, ranks, capacity) -> gpurun_out/$TAG/<case>_<ranks>r_b<cap>.json. Each run under its own
# time limit; the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
TAG=${1:-leafcap}; shift
O=gpurun_out/$TAG; mkdir -p "$O"
for spec in "$@"; do
    IFS=: read -r init n ranks caps <<< "$spec"
    for cap in ${caps//,/ }; do
        SPHX_BUCKET_FOCUS=$cap SPHX_BENCH_SHARED_GPU=1 timeout -k 10 ${RUN_TIMEOUT:-400} python3 bench.py --gpus "$ranks" \
            --init "$init" -n "$n" --steps ${STEPS:-4} --warmup 2 > "$O/${init}_${ranks}r_b${cap}.json" 2> "$O/${init}_${ranks}r_b${cap}.err" \
            || { tail -5 "$O/${init}_${ranks}r_b${cap}.err"; exit 1; }
        echo "$init -n $n ranks $ranks cap $cap: $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'])" "$O/${init}_${ranks}r_b${cap}.json") ms/step"
    done
done
