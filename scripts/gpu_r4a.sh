#!/bin/bash
# round 4, first GPU pass: full GPU test suite, default bench, Evrard kernel table, gravity LDS counters
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4a; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests -m gpu -q --maxfail=15 --timeout 150 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests.log | tail -2; grep FAILED $O/tests.log | head -15
[ $rc -gt 1 ] && { echo "pytest rc $rc: stopping"; tail -30 $O/tests.log; exit 1; }
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"evrard_ms_per_step": [0-9.]*' $O/bench.json
timeout -k 10 200 python3 scripts/grav_stats.py > $O/grav_stats.txt 2>&1 || { tail -20 $O/grav_stats.txt; exit 1; }
cat $O/grav_stats.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/evrard -o run -- \
    python3 bench.py --init evrard -n 200 --steps 3 --warmup 2 > $O/evrard.log 2>&1 || { tail -5 $O/evrard.log; exit 1; }
python3 scripts/kernel_table.py $O/evrard/run_kernel_stats.csv 5 > $O/evrard_kernels.md; head -24 $O/evrard_kernels.md
timeout -s KILL 200 rocprofv3 --kernel-include-regex "gravity(P2P|M2P)Kernel" --pmc SQ_WAVES SQ_LDS_BANK_CONFLICT \
    SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $O/pmc -o run -- \
    python3 bench.py --init evrard -n 200 --steps 1 --warmup 1 > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
python3 - <<'PY'
import csv, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open("gpurun_out/r4a/pmc/run_counter_collection.csv")):
    agg[r["Kernel_Name"][:40]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, a in agg.items():
    w = max(a["SQ_WAVES"], 1); c = max(a["SQ_WAVE_CYCLES"], 1)
    print(k, "waves", int(w), "bank conflicts/wave %.0f" % (a["SQ_LDS_BANK_CONFLICT"] / w),
          "LDS/wave %.0f" % (a["SQ_INSTS_LDS"] / w), "wait-inst %.2f" % (a["SQ_WAIT_INST_ANY"] / c),
          "valu-active %.2f" % (a["SQ_ACTIVE_INST_VALU"] / c))
PY
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/e100 -o run -- \
    python3 bench.py --init evrard -n 100 --steps 5 --warmup 3 > $O/e100.log 2>&1 || { tail -5 $O/e100.log; exit 1; }
python3 scripts/gpu_busy.py $O/e100/run_kernel_trace.csv 4 > $O/e100_busy.txt; head -3 $O/e100_busy.txt
python3 scripts/step_sequence.py $O/e100/run_kernel_trace.csv -2 > $O/e100_seq.txt; tail -12 $O/e100_seq.txt
timeout -k 10 200 python3 scripts/host_profile.py --init evrard -n 100 --steps 20 --top 60 > $O/e100_host.txt 2>&1 \
    || { tail -5 $O/e100_host.txt; exit 1; }
grep "ms/step" $O/e100_host.txt
