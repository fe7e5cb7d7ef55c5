# A/B of build variants and environment settings by kernel time (as ab_kernels.sh):
#   bash scripts/ab_kernels_env.sh TAG "bench args" "name:variant:ENV=VAL ..." ...  (variant "default" = main build)
set -o pipefail
TAG=$1; ARGS=$2; shift 2
O=gpurun_out/abk_$TAG; mkdir -p "$O"
export TMPDIR=/tmp
for r in 1 2; do
  for spec in "$@"; do
    name=${spec%%:*}; rest=${spec#*:}; v=${rest%%:*}; envs=${rest#*:}
    if [ "$v" = default ]; then unset SPHX_HIP_VARIANT; else export SPHX_HIP_VARIANT=$v; fi
    timeout -k 10 300 env $envs rocprofv3 --kernel-trace --output-format csv -d "$O/${name}_$r" -o run -- \
        python3 bench.py $ARGS > "$O/${name}_$r.log" 2>&1 || exit 1
  done
done
python3 - "$O" > "$O/table.txt" <<'PY'
import csv, collections, glob, sys, os
O = sys.argv[1]
res = {}
for f in sorted(glob.glob(f"{O}/*_[12]/run_kernel_trace.csv")):
    t = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        t[r["Kernel_Name"].split("(")[0][:60]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    res[os.path.basename(os.path.dirname(f))] = t
names = set()
for t in res.values():
    names |= {n for n, x in t.items() if sum(x) > 5}
print("kernel | " + " | ".join(res))
for n in sorted(names, key=lambda n: -sum(sum(t.get(n, [])) for t in res.values())):
    print(f"{n} | " + " | ".join(f"{sum(t.get(n, [])) / max(len(t.get(n, [])), 1):.3f}" for t in res.values()))
PY
cat "$O/table.txt"
