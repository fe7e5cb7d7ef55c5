#!/bin/bash
# Counter passes (one rocprofv3 run each) over the main neighbor-search kernel on a case's steady state
# (scripts/search_timing.py): usage bash scripts/pmc_search.sh TAG [search_timing args] -> gpurun_out/pmcs_TAG/p*/
set -o pipefail
TAG=$1; shift
R=$(pwd)
OUT=$R/gpurun_out/pmcs_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
P2="SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD"
i=0
for P in "$P1" "$P2"; do
  i=$((i + 1))
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-include-regex findNeighborsKernel --output-format csv \
      -d "$OUT/p$i" -o run -- python3 "$R/scripts/search_timing.py" "$@" > "$OUT/p$i.log" 2>&1 || exit $?
done
python3 - "$OUT" <<'PY'
import csv, collections, glob, sys
agg = collections.defaultdict(float)
for f in glob.glob(sys.argv[1] + "/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
w = max(agg.get("SQ_WAVES", 1), 1)
for k in sorted(agg):
    print(f"{k:24s} {agg[k]:16.0f}  per wave {agg[k] / w:10.1f}")
PY
