#!/usr/bin/env python3
"""Print a kernel timeline (start offset, duration) from a rocprofv3 kernel_trace.csv, optionally filtered by a
regex, to check stream overlap. usage: python scripts/trace_kernels.py TRACE.csv [REGEX] [LAST_N]"""

import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rx = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
last = int(sys.argv[3]) if len(sys.argv) > 3 else 40
rows = [r for r in rows if rx is None or rx.search(r["Kernel_Name"])]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-last:]
t0 = int(rows[0]["Start_Timestamp"]) if rows else 0
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:10.1f} us  {(e - s) / 1e3:9.1f} us  q{r.get('Queue_Id', '?'):>3}  {r['Kernel_Name'][:70]}")
