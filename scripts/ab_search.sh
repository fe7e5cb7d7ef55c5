# A/B of search build variants (scripts/search_timing.py) on Sedov -n 400 and Evrard -n 200, alternating:
#   bash scripts/ab_search.sh TAG variant1 variant2 ...   ("default" = the main build) -> gpurun_out/abs_TAG/
set -o pipefail
TAG=$1; shift
O=gpurun_out/abs_$TAG; mkdir -p "$O"
for r in 1 2; do
  for v in "$@"; do
    if [ "$v" = default ]; then unset SPHX_HIP_VARIANT; else export SPHX_HIP_VARIANT=$v; fi
    timeout -k 10 200 python3 scripts/search_timing.py --init sedov -n 400 --presteps 1 --reps 5 >> "$O/sedov.log" 2>&1 || exit 1
  done
done
grep -h "search " "$O"/*.log
