#!/usr/bin/env python3
"""Ordered kernel sequence of one time step from a rocprofv3 kernel trace (a step starts at its SFC key kernel):
start offset, idle gap before the kernel, duration and name, plus the torch (at::native / rocclr) kernels of the
step counted by name. usage: python scripts/step_sequence.py TRACE.csv [STEP=-2] [MARKER=computeKeysKernel]"""
import csv
import re
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    which = int(sys.argv[2]) if len(sys.argv) > 2 else -2
    marker = re.compile(sys.argv[3] if len(sys.argv) > 3 else "computeKeysKernel")
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    starts = [s for s, e, n in ev if marker.search(n)]
    t0 = starts[which]
    t1 = starts[which + 1] if which + 1 < len(starts) and which != -1 else max(e for s, e, n in ev) + 1
    step = [x for x in ev if t0 <= x[0] < t1]
    prev_end = step[0][0]
    torch_k = {}
    busy = 0
    print(f"{'start us':>9} {'gap us':>8} {'dur us':>8}  kernel")
    for s, e, n in step:
        gap = max(0, s - prev_end)
        name = n.split("(")[0].replace("void ", "")[:90]
        print(f"{(s - t0) / 1e3:9.1f} {gap / 1e3:8.1f} {(e - s) / 1e3:8.1f}  {name}")
        busy += e - max(s, prev_end) if e > prev_end else 0
        prev_end = max(prev_end, e)
        if name.startswith("at::") or "rocclr" in name or "native" in name:
            torch_k[name[:70]] = torch_k.get(name[:70], 0) + 1
    span = step[-1][1] - t0
    print(f"step span {span / 1e3:.1f} us, busy {100.0 * busy / span:.1f} %, {len(step)} kernels, "
          f"{sum(torch_k.values())} torch/runtime kernels")
    for k, c in sorted(torch_k.items(), key=lambda kv: -kv[1]):
        print(f"  {c:3d} x {k}")


if __name__ == "__main__":
    main()
