# A/B of build variants by kernel time: one kernel trace of a short bench run per variant, twice, alternating.
#   bash scripts/ab_kernels.sh TAG "bench args" variant1 variant2 ...  ("default" = the main build)
#   -> gpurun_out/abk_TAG/<variant>_<run>/ and a per-kernel table (ms per call) in gpurun_out/abk_TAG/table.txt
set -o pipefail
TAG=$1; ARGS=$2; shift 2
O=gpurun_out/abk_$TAG; mkdir -p "$O"
export TMPDIR=/tmp
for r in 1 2; do
  for v in "$@"; do
    if [ "$v" = default ]; then unset SPHX_HIP_VARIANT; else export SPHX_HIP_VARIANT=$v; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/${v}_$r" -o run -- \
        python3 bench.py $ARGS > "$O/${v}_$r.log" 2>&1 || exit 1
  done
done
python3 - "$O" "$@" > "$O/table.txt" <<'PY'
import csv, collections, glob, sys
O, variants = sys.argv[1], sys.argv[2:]
res = {}
for v in variants:
    for f in sorted(glob.glob(f"{O}/{v}_*/run_kernel_trace.csv")):
        t = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            t[r["Kernel_Name"].split("(")[0][:60]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
        res[f] = (v, t)
names = set()
for v, t in res.values():
    names |= {n for n, x in t.items() if sum(x) > 5}
print("kernel | " + " | ".join(f"{v} run{k}" for k, (v, t) in enumerate(res.values())))
for n in sorted(names, key=lambda n: -sum(sum(t.get(n, [])) for v, t in res.values())):
    cells = []
    for v, t in res.values():
        x = t.get(n, [])
        cells.append(f"{sum(x) / max(len(x), 1):.3f}")
    print(f"{n} | " + " | ".join(cells))
PY
cat "$O/table.txt"
