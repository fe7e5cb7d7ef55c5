# search time by elimination (timing variants built with SPHX_NS_TIMING_*; lists unusable, one round, ICs):
#   bash scripts/search_breakdown.sh TAG [search_timing args] -> gpurun_out/sbd_TAG.log
set -o pipefail
TAG=$1; shift
O=gpurun_out/sbd_$TAG.log
for v in default tnotouch tnocand tnotest default; do
  if [ "$v" = default ]; then unset SPHX_HIP_VARIANT; else export SPHX_HIP_VARIANT=$v; fi
  timeout -k 10 200 python3 scripts/search_timing.py --no-iterate --reps 5 "$@" >> "$O" 2>&1 || exit 1
done
grep -h "search " "$O"
