#!/usr/bin/env python3
"""per-kernel instruction statistics of a device assembly file (hipcc --cuda-device-only -S): transcendental and
VALU instruction counts of the kernels whose names match REGEX

usage: python scripts/asm_stats.py FILE.s [REGEX]
"""
import re
import sys

s = open(sys.argv[1]).read()
rx = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
valu = re.compile(r"^\s+v_", re.M)
for m in re.finditer(r"^(_ZN4sphx3hip[^\n:]*):[^\n]*\n(.*?)s_endpgm", s, re.S | re.M):
    name, body = m.group(1), m.group(2)
    if not rx.search(name):
        continue
    cnt = {k: len(re.findall(k, body)) for k in ("v_exp_f32", "v_log_f32", "v_sin_f32", "v_cos_f32", "v_rcp_f32")}
    print(f"{name[:64]:66s} " + " ".join(f"{k[2:5]} {v:3d}" for k, v in cnt.items()) +
          f" valu {len(valu.findall(body)):5d}")
