#!/bin/bash
# counter passes for the gravity evaluation kernels (grav_micro, Evrard -n 200)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/pmc_grav; mkdir -p $OUT; export TMPDIR=/tmp
B="python3 scripts/grav_micro.py -n 200 -k 2"
RX="gravityP2PKernel|gravityM2PKernel|gravityListKernel"
run() { timeout -s KILL 150 rocprofv3 --kernel-include-regex "$RX" --pmc "$@" --output-format csv -d $OUT/p$N -o run -- $B > $OUT/p$N.log 2>&1 || { echo "pass $N failed"; tail -3 $OUT/p$N.log; exit 1; }; N=$((N+1)); }
N=1
run SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
run SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INST_CYCLES_VMEM_RD
run TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE
python3 - $OUT <<'PY'
import csv, sys, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, a in agg.items():
    w = max(a.get("SQ_WAVES", 1), 1); cyc = max(a.get("SQ_WAVE_CYCLES", 1), 1)
    print(k)
    for c in sorted(a):
        v = a[c]
        extra = f"  ({v / cyc:.3f} of wave-cycles)" if c.startswith(("SQ_WAIT", "SQ_ACTIVE")) else (f"  ({v / w:.1f} per wave)" if c.startswith("SQ_INST") else "")
        print(f"   {c:32s} {v:16.0f}{extra}")
PY
