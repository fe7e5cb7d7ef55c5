"""Per-wave counter table from rocprofv3 --pmc csv outputs: python scripts/pmc_table.py DIR [DIR ...] (each DIR holds
p*/run_counter_collection.csv). Counters are summed over dispatches and divided by SQ_WAVES."""
import collections
import csv
import glob
import sys


def load(d):
    agg = collections.defaultdict(float)
    waves = 0.0
    for f in sorted(glob.glob(f"{d}/p*/run_counter_collection.csv")):
        part = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            part[r["Counter_Name"]] += float(r["Counter_Value"])
        waves = part.get("SQ_WAVES", waves)
        for k, v in part.items():
            if k != "SQ_WAVES":
                agg[k] = v
    return waves, agg


def main():
    cols = {}
    for d in sys.argv[1:]:
        cols[d] = load(d)
    keys = sorted({k for _, a in cols.values() for k in a})
    print("| counter (per wave) | " + " | ".join(d.rstrip("/").split("/")[-1] for d in cols) + " |")
    print("|---" * (len(cols) + 1) + "|")
    for k in keys:
        print(f"| {k} | " + " | ".join(f"{a.get(k, 0) / max(w, 1):.0f}" for w, a in cols.values()) + " |")


if __name__ == "__main__":
    main()
