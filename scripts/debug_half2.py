#!/usr/bin/env python3
"""debug: NaN census after Evrard steps"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sphexa_amd.app.simulation import Simulation  # noqa: E402
from sphexa_amd.ops import gravity as G  # noqa: E402

for n in [int(v) for v in sys.argv[1:]]:
    sim = Simulation("evrard", n=n)
    d = sim.d
    for k in range(2):
        sim.step()
        bad = {}
        for f in ("x", "h", "ax", "vx", "u", "rho"):
            try:
                bad[f] = int(torch.isnan(d[f]).sum())
            except Exception:
                pass
        print(f"n={n} step {k}: NaN {bad} egrav {d.egrav:.6e} caps {G._CAPS}", flush=True)
