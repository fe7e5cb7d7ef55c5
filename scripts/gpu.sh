#!/bin/bash
# One parameterised runner for the GPU box (used through gpurun). Every GPU step has its own time limit and the
# script stops at the first failing step. Output goes to gpurun_out/<TAG>/.
#
#   bash scripts/gpu.sh tests TAG [pytest paths...]      gpu-marked tests in one process
#   bash scripts/gpu.sh bench TAG [bench.py args...]     one bench.py run -> TAG/bench.json
#   bash scripts/gpu.sh busy TAG [bench.py args...]      kernel trace + stats + GPU-busy table (scripts/gpu_busy.py)
#   bash scripts/gpu.sh pmc TAG REGEX "C1 C2 .." [bench.py args...]   one counter pass over kernels matching REGEX
#   bash scripts/gpu.sh avail TAG                        rocprofv3 counter list
#   bash scripts/gpu.sh shared TAG N [bench.py args...]  N ranks sharing cuda:0 over gloo (multi-rank rehearsal)
#
# Several commands can be chained with && in one gpurun call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
export TMPDIR=/tmp
CMD=$1; TAG=$2; shift 2
O=gpurun_out/$TAG; mkdir -p "$O"
case "$CMD" in
tests)
    timeout -k 10 ${GPU_TEST_TIMEOUT:-900} python -u -m pytest ${@:-tests} -m gpu -x -v --timeout 120 \
        --timeout-method thread > "$O/tests.log" 2>&1
    rc=$?; tail -3 "$O/tests.log"; exit $rc ;;
bench)
    timeout -k 10 ${BENCH_TIMEOUT:-600} python3 bench.py "$@" > "$O/bench.json" 2> "$O/bench.err"
    rc=$?; cat "$O/bench.json"; [ $rc -ne 0 ] && tail -20 "$O/bench.err"; exit $rc ;;
busy)
    timeout -k 10 ${BENCH_TIMEOUT:-600} rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o run -- \
        python3 bench.py "$@" > "$O/kt.log" 2>&1 || { tail -20 "$O/kt.log"; exit 1; }
    python3 scripts/gpu_busy.py "$O/kt/run_kernel_trace.csv" ${BUSY_STEPS:-3} computeKeys > "$O/busy.txt" && head -40 "$O/busy.txt" ;;
pmc)
    # PROG overrides the profiled program (default bench.py), e.g. PROG="python3 scripts/grav_micro.py"
    RX=$1; CTR=$2; shift 2
    P=${PMC_PASS:-p}
    if [ -s gpurun_out/avail/avail.txt ]; then
        # counters this device does not list are dropped (an unknown name fails the whole pass)
        KEEP=""; for c in $CTR; do b=${c%_sum}; if grep -qw -- "$b" gpurun_out/avail/avail.txt; then KEEP="$KEEP $c";
            else echo "dropping counter $c (not listed)"; fi; done; CTR=$KEEP
    fi
    timeout -s KILL ${PMC_TIMEOUT:-240} rocprofv3 --kernel-include-regex "$RX" --pmc $CTR --output-format csv \
        -d "$O/$P" -o run -- ${PROG:-python3 bench.py} "$@" > "$O/$P.log" 2>&1 || { tail -20 "$O/$P.log"; exit 1; }
    python3 scripts/pmc_table.py "$O/$P/run_counter_collection.csv" > "$O/$P.txt" && cat "$O/$P.txt" ;;
avail)
    timeout -s KILL 60 rocprofv3 -L > "$O/avail.txt" 2>&1; echo "avail rc $?"; wc -l "$O/avail.txt" ;;
shared)
    N=$1; shift
    SPHX_BENCH_SHARED_GPU=1 timeout -k 10 ${BENCH_TIMEOUT:-600} python3 bench.py --gpus $N "$@" > "$O/bench.json" \
        2> "$O/bench.err"
    rc=$?; cat "$O/bench.json"; [ $rc -ne 0 ] && tail -20 "$O/bench.err"; exit $rc ;;
*)
    echo "unknown command $CMD"; exit 2 ;;
esac
