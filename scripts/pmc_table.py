"""Per-kernel counter table from rocprofv3 --pmc csv output(s): python scripts/pmc_table.py FILE.csv [FILE.csv ...].
Counters are summed over dispatches; per-wave values are given where SQ_WAVES was collected in the same file.
Several files (separate passes of one run) are merged per kernel."""
import collections
import csv
import sys


def main():
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    calls = collections.defaultdict(set)
    for f in sys.argv[1:]:
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:80]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            calls[k].add(r.get("Dispatch_Id", ""))
    for k, a in sorted(agg.items()):
        w = a.get("SQ_WAVES", 0)
        print(f"{k}  (dispatches {len(calls[k])})")
        for c in sorted(a):
            v = a[c]
            extra = f"   {v / w:14.1f} per wave" if w and c != "SQ_WAVES" else ""
            print(f"   {c:34s} {v:18.0f}{extra}")


if __name__ == "__main__":
    main()
