#!/usr/bin/env python3
"""GPU-busy fraction of the timed steps from a rocprofv3 kernel trace: union of kernel execution intervals divided by
the wall span, over the steps after the first SKIP ones (a step starts at its SFC key kernel), plus the largest idle
gaps (host-side work / syncs between kernels) and a per-step table.

usage: python scripts/gpu_busy.py TRACE.csv [SKIP=1] [MARKER=computeKeysKernel]
"""

import csv
import re
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    skip = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    marker = re.compile(sys.argv[3] if len(sys.argv) > 3 else "computeKeysKernel")
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    starts = [s for s, e, n in ev if marker.search(n)]
    if len(starts) <= skip:
        print("not enough steps in the trace")
        return
    t0 = starts[skip]
    ev = [x for x in ev if x[0] >= t0]
    t1 = max(e for s, e, n in ev)
    busy, cur_s, cur_e = 0, None, None
    gaps = []
    for s, e, n in ev:
        if cur_e is None:
            cur_s, cur_e, prev = s, e, n
            continue
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, prev, n))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        prev = n
    busy += cur_e - cur_s
    span = t1 - t0
    nsteps = len(starts) - skip
    print(f"steps {nsteps}, span {span / 1e6:.2f} ms ({span / 1e6 / nsteps:.2f} ms/step), kernel-busy {busy / 1e6:.2f} ms "
          f"-> GPU busy {100.0 * busy / span:.1f} %, {len(ev) / nsteps:.0f} kernels/step")
    per = {}
    for s_, e_, n_ in ev:
        k = n_.split("(")[0].replace("void ", "")[:70]
        c, t = per.get(k, (0, 0))
        per[k] = (c + 1, t + e_ - s_)
    print("kernel time per step (timed window):")
    for k, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][1])[:14]:
        print(f"  {t / 1e6 / nsteps:8.3f} ms  {c / nsteps:5.1f} calls  {k}")
    gaps.sort(reverse=True)
    tot = sum(g for g, _, _ in gaps)
    print(f"idle {tot / 1e6:.2f} ms in {len(gaps)} gaps; largest:")
    for g, a, b in gaps[:12]:
        print(f"  {g / 1e3:8.1f} us  after {a[:60]}  before {b[:60]}")


if __name__ == "__main__":
    main()
