"""Markdown table of a rocprofv3 kernel-stats csv, per time step: python scripts/kernel_table.py STATS.csv STEPS [TOP]"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    steps = float(sys.argv[2])
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"kernel time per step: {tot / 1e6 / steps:.2f} ms ({steps:g} profiled steps incl. warmup)")
    print("| kernel | calls/step | ms/step | % |")
    print("|---|---|---|---|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        name = r["Name"].split("(")[0].replace("void ", "")[:80]
        print(f"| {name} | {float(r['Calls']) / steps:.1f} | {float(r['TotalDurationNs']) / 1e6 / steps:.3f} | "
              f"{100 * float(r['TotalDurationNs']) / tot:.1f} |")


if __name__ == "__main__":
    main()
