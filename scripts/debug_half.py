#!/usr/bin/env python3
"""debug: gravity statistics and energy for repeated evaluations, with the default and grown slab caps"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_gravity import _setup  # noqa: E402

from sphexa_amd.ops import gravity as G  # noqa: E402


def run(tag, args, n):
    acc = [torch.zeros(n, dtype=torch.float32, device="cuda") for _ in range(3)]
    st = {}
    e = G.compute_gravity(*args, *acc, stats=st)
    a = torch.sqrt(acc[0] ** 2 + acc[1] ** 2 + acc[2] ** 2)
    print(f"{tag:>28}: egrav {e:.9e} |a| max {float(a.max()):.4e} nan {int(torch.isnan(a).sum())} caps {G._CAPS} "
          f"p2p {st['p2p']} m2p {st['m2p']} fb {st['fallback']}", flush=True)
    return acc


n = 50000
box, ot, x, y, z, m, h = _setup(n, torch.device("cuda", 0))
c, mp = G.upsweep(ot, x, y, z, m, box, 0.5)
args = (ot, c, mp, 0, n, x, y, z, h, m, 1.0)
run("plummer first", args, n)
run("plummer second", args, n)
caps = dict(G._CAPS)
for cm, cl in ((caps["m"] + 64, caps["l"]), (caps["m"], caps["l"] + 64), (3008, 1472)):
    G._CAPS["m"], G._CAPS["l"] = cm, cl
    run(f"plummer caps {cm},{cl}", args, n)
G._CAPS.update(caps)
G.TEST_CAPS = (256, 64)
run("plummer TEST_CAPS 256,64", args, n)
G.TEST_CAPS = None
G.TEST_FRONT_CAP = 16
run("plummer TEST_FRONT_CAP 16", args, n)
G.TEST_FRONT_CAP = 0
if len(sys.argv) > 2:
    sys.exit(0)

from sphexa_amd.app.simulation import Simulation  # noqa: E402

sim = Simulation("evrard", n=int(sys.argv[1]) if len(sys.argv) > 1 else 50)
sim.step()
d, dom = sim.d, sim.domain
mh = sim.propagator.gravity
mh.upsweep(d, dom)
s, e = dom.start_index(), dom.end_index()
args = (dom.octree, mh.centers, mh.multipoles, s, e, d["x"], d["y"], d["z"], d["h"], d["m"], d.g)
run("evrard first", args, d.size)
run("evrard second", args, d.size)
