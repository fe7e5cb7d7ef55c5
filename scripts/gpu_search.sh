#!/bin/bash
# neighbor-search changes: parity/spill/split tests, then kernel tables of Evrard -n 100 and Noh -n 300
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-search}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cases.py -m gpu -q --timeout 150 \
    --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -4 $O/tests.log; [ $rc -eq 0 ] || { grep FAILED $O/tests.log; exit $rc; }
prof() { # tag args...
  local tag=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o run -- \
      python3 bench.py --steps 3 --warmup 2 "$@" > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -5 $O/$tag.log; return 1; }
  python3 scripts/kernel_table.py $O/$tag/run_kernel_stats.csv 3 > $O/$tag.md
  echo "== $tag"; grep -i "neighbor\|total\|kernel time" $O/$tag.md | head -6
}
prof e100 --init evrard -n 100 && prof noh300 --init noh -n 300
