#!/bin/bash
# gravity kernel times: in-tree build + variants given, then the _old worktree (previous commit), Evrard -n 200
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_grav_variants.sh "$@" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/gv; cd _old || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/old -o run -- \
    python3 scripts/grav_micro.py -n ${GRAV_N:-200} -k 5 > $O/old.log 2>&1 || { echo "old failed"; tail -5 $O/old.log; exit 1; }
grep "evaluation" $O/old.log
python3 - $O/old/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "gravityP2P" in n or "gravityM2P" in n or "gravityList" in n:
        print(f"           old {n.split('(')[0][-22:]:>22} {float(r['AverageNs']) / 1e6:7.3f} ms x {r['Calls']}")
PY
