#!/bin/bash
# per-kernel gravity times of the in-tree build and the HIP variants given (_native/variants/TAG), Evrard -n 200
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/gv; mkdir -p $O; export TMPDIR=/tmp
for tag in default "$@"; do
  if [ "$tag" = default ]; then unset SPHX_HIP_VARIANT; else export SPHX_HIP_VARIANT=$tag; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o run -- \
      python3 scripts/grav_micro.py -n ${GRAV_N:-200} -k 5 > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -5 $O/$tag.log; exit 1; }
  grep "evaluation" $O/$tag.log
  python3 - $O/$tag/run_kernel_stats.csv $tag <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "gravityP2P" in n or "gravityM2P" in n or "gravityList" in n:
        print(f"  {sys.argv[2]:>12} {n.split('(')[0][-22:]:>22} {float(r['AverageNs']) / 1e6:7.3f} ms x {r['Calls']}")
PY
done
