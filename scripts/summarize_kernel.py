#!/usr/bin/env python3
"""Summarize scripts/profile_kernel.sh output: kernel time table + every collected counter per matching kernel,
normalized per wave and per wave-cycle. usage: python scripts/summarize_kernel.py gpurun_out/kprof_TAG"""

import collections
import csv
import glob
import os
import sys


def main(d):
    p = os.path.join(d, "stats", "run_kernel_stats.csv")
    if os.path.exists(p):
        print("| kernel | calls | total ms | avg us | % |\n|---|---|---|---|---|")
        for r in list(csv.DictReader(open(p)))[:15]:
            print(f"| {r['Name'][:80]} | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.2f} | "
                  f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.2f} |")
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    meta = {}
    for f in sorted(glob.glob(os.path.join(d, "pmc*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:70]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            meta[k] = {x: r.get(x) for x in ("VGPR_Count", "Accum_VGPR_Count", "SGPR_Count", "LDS_Block_Size",
                                             "Workgroup_Size", "Grid_Size")}
    for k, v in agg.items():
        print(f"\n### {k}\n\n{meta[k]}\n")
        w = max(v.get("SQ_WAVES", 1), 1)
        cyc = max(v.get("SQ_WAVE_CYCLES", 1), 1)
        print("| counter | total | per wave | per wave-cycle |\n|---|---|---|---|")
        for c in sorted(v):
            print(f"| {c} | {v[c]:.4g} | {v[c] / w:.4g} | {v[c] / cyc:.4f} |")


if __name__ == "__main__":
    main(sys.argv[1])
