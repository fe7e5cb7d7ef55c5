#!/bin/bash
# small per-rank sizes (the 8-GPU shares): non-verbose bench times + GPU-busy traces of Evrard -n 100 and Sedov -n 200
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-small}
for c in "evrard 100" "sedov 200"; do
  set -- $c
  timeout -k 10 200 python -u bench.py --init $1 -n $2 --steps 20 --warmup 3 > gpurun_out/${TAG}_$1$2.json 2>&1 || { tail -5 gpurun_out/${TAG}_$1$2.json; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/${TAG}_$1$2.json | sed "s/^/$1 -n $2 /"
  bash scripts/profile_busy.sh ${TAG}_$1$2 --init $1 -n $2 | head -3 || exit 1
done
