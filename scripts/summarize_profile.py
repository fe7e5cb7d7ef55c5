#!/usr/bin/env python3
"""Turn a scripts/profile_gpu.sh output directory (rocprofv3 csv) into a markdown summary for profiles/.

usage: python scripts/summarize_profile.py gpurun_out/prof_n200 > profiles/<name>.md
"""

import collections
import csv
import os
import sys


def kernel_stats(d):
    p = os.path.join(d, "stats", "run_kernel_stats.csv")
    if not os.path.exists(p):
        return []
    rows = list(csv.DictReader(open(p)))
    out = ["| kernel | calls | total ms | avg us | % |", "|---|---|---|---|---|"]
    for r in rows[:30]:
        out.append(f"| {r['Name'][:90]} | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.2f} | "
                   f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.2f} |")
    return out


def pmc(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    meta = {}
    for sub in ("pmc1", "pmc2"):
        p = os.path.join(d, sub, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:60]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            meta[k] = (r.get("VGPR_Count"), r.get("LDS_Block_Size"))
    out = ["| kernel | waves | VALU/wave | VMEM rd/wave | LDS/wave | active | wait(any) | wait(inst) | L2 hit | "
           "fetch MB | LDS bank conf |", "|---|---|---|---|---|---|---|---|---|---|---|"]
    rows = []
    for k, v in agg.items():
        cyc = v.get("SQ_WAVE_CYCLES", 0)
        w = max(v.get("SQ_WAVES", 0), 1)
        if cyc <= 0 or w < 100:
            continue
        hit, miss = v.get("TCC_HIT_sum", 0), v.get("TCC_MISS_sum", 0)
        rows.append((v.get("SQ_INSTS_VALU", 0), f"| {k} | {w:.0f} | {v.get('SQ_INSTS_VALU', 0) / w:.0f} | "
                     f"{v.get('SQ_INSTS_VMEM_RD', 0) / w:.0f} | {v.get('SQ_INSTS_LDS', 0) / w:.0f} | "
                     f"{v.get('SQ_ACTIVE_INST_ANY', 0) / cyc:.2f} | {v.get('SQ_WAIT_ANY', 0) / cyc:.2f} | "
                     f"{v.get('SQ_WAIT_INST_ANY', 0) / cyc:.2f} | {hit / max(hit + miss, 1):.3f} | "
                     f"{v.get('FETCH_SIZE', 0) / 1024:.0f} | {v.get('SQ_LDS_BANK_CONFLICT', 0):.0f} |"))
    rows.sort(key=lambda t: -t[0])
    return out + [r for _, r in rows]


def bench(d):
    p = os.path.join(d, "bench.log")
    if not os.path.exists(p):
        return []
    return ["```"] + [l.rstrip() for l in open(p) if l.startswith(("{", "# substep", "# max", "# gravity"))] + ["```"]


def main():
    d = sys.argv[1]
    print(f"# rocprofv3 summary of `{d}`\n")
    print("## bench (substep timings, device-synchronized)\n")
    print("\n".join(bench(d)))
    print("\n## kernel trace statistics (--kernel-trace --stats)\n")
    print("\n".join(kernel_stats(d)))
    print("\n## hardware counters per kernel (--pmc, summed over dispatches)\n")
    print("active / wait = SQ_ACTIVE_INST_ANY / SQ_WAIT_ANY / SQ_WAIT_INST_ANY over SQ_WAVE_CYCLES; FETCH_SIZE is "
          "half the real bytes on gfx950 for wide loads (MI355X_MICROARCH.md)\n")
    print("\n".join(pmc(d)))


if __name__ == "__main__":
    main()
