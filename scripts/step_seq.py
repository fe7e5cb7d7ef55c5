#!/usr/bin/env python3
"""one step's kernel sequence from a rocprofv3 kernel trace: start offset, gap to the previous kernel's end (negative:
overlap on another stream), duration (us) and name.

usage: python scripts/step_seq.py TRACE.csv [STEP=-2] [FILTER_REGEX]
"""
import csv
import re
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    step = int(sys.argv[2]) if len(sys.argv) > 2 else -2
    rx = re.compile(sys.argv[3]) if len(sys.argv) > 3 else None
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                 r["Kernel_Name"].split("(")[0].replace("void ", "").replace("sphx::hip::", "")[:60]) for r in rows)
    starts = [s for s, e, n in ev if "computeKeys" in n]
    t0, t1 = starts[step], starts[step + 1] if step + 1 < len(starts) and step != -1 else ev[-1][1] + 1
    cur = t0
    for s, e, n in ev:
        if t0 <= s < t1:
            if rx is None or rx.search(n):
                print(f"{(s - t0) / 1e3:9.1f} {(s - cur) / 1e3:8.1f} {(e - s) / 1e3:8.1f}  {n}")
            cur = max(cur, e)


if __name__ == "__main__":
    main()
