#!/usr/bin/env python3
"""ms/step of bench.py JSON lines written by scripts/gpu.sh bench (gpurun_out/<TAG>/bench.json)

usage: python scripts/bench_table.py TAG [TAG ...]
"""
import json
import os
import sys

for tag in sys.argv[1:]:
    p = os.path.join("gpurun_out", tag, "bench.json")
    try:
        lines = [ln for ln in open(p).read().splitlines() if ln.startswith('{"metric')]
        d = json.loads(lines[-1])
        print(f"{tag:24s} {d['ms_per_step']:9.3f} ms/step  {d['value'] / 1e6:9.1f} M/s  {d['config']['model']}")
    except (OSError, IndexError, ValueError) as e:
        print(f"{tag:24s} (no result: {e.__class__.__name__})")
