set -o pipefail
O=gpurun_out/abenv; mkdir -p $O
for r in 1 2; do
  for cfg in "base:" "prio:SPHX_GRAV_PRIORITY=-1" "lfirst:SPHX_GRAV_LISTS_FIRST=1"; do
    tag=${cfg%%:*}; env=${cfg#*:}
    timeout -k 10 300 env $env python3 bench.py --init evrard -n 200 --steps 10 --warmup 3 > $O/${tag}_$r.json 2> $O/${tag}_$r.err || exit 1
    echo "$tag $r $(python3 -c "import json;print(json.load(open('$O/${tag}_$r.json'))['ms_per_step'])")"
  done
done
