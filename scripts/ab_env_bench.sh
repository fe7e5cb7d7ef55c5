# A/B of environment settings on one bench case, two alternating runs each:
#   bash scripts/ab_env_bench.sh TAG "bench args" "name:ENV=VAL ..." ...   -> gpurun_out/abenv_TAG/
set -o pipefail
TAG=$1; ARGS=$2; shift 2
O=gpurun_out/abenv_$TAG; mkdir -p $O
for r in 1 2; do
  for cfg in "$@"; do
    tag=${cfg%%:*}; env=${cfg#*:}
    timeout -k 10 300 env $env python3 bench.py $ARGS > $O/${tag}_$r.json 2> $O/${tag}_$r.err || exit 1
    echo "$tag $r $(python3 -c "import json;print(round(json.load(open('$O/${tag}_$r.json'))['ms_per_step'], 3))")"
  done
done
