"""Per-kernel counter table (summed over dispatches, per wave) + kernel time share from a prof_step.sh run:
python scripts/pmc_kernels.py gpurun_out/TAG"""
import collections
import csv
import sys


def main():
    d = sys.argv[1]
    stats = list(csv.DictReader(open(f"{d}/kt/run_kernel_stats.csv")))
    tot = sum(float(r["TotalDurationNs"]) for r in stats)
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f"{d}/pmc/run_counter_collection.csv")):
        agg[r["Kernel_Name"][:60]][r["Counter_Name"]] += float(r["Counter_Value"])
    print("| kernel | calls | ms/call | % | VALU/wave | SALU/wave | LDS/wave | VMEM rd/wave | issue-active | wait-inst |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for r in sorted(stats, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
        name = r["Name"][:60]
        a = agg.get(name, {})
        w = max(a.get("SQ_WAVES", 0), 1)
        cyc = max(a.get("SQ_WAVE_CYCLES", 0), 1)
        print(f"| {r['Name'][:70]} | {r['Calls']} | {float(r['AverageNs']) / 1e6:.2f} | "
              f"{100 * float(r['TotalDurationNs']) / tot:.1f} | {a.get('SQ_INSTS_VALU', 0) / w:.0f} | "
              f"{a.get('SQ_INSTS_SALU', 0) / w:.0f} | {a.get('SQ_INSTS_LDS', 0) / w:.0f} | "
              f"{a.get('SQ_INSTS_VMEM_RD', 0) / w:.0f} | {a.get('SQ_ACTIVE_INST_ANY', 0) / cyc:.2f} | "
              f"{a.get('SQ_WAIT_INST_ANY', 0) / cyc:.2f} |")


if __name__ == "__main__":
    main()
