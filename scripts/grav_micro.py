#!/usr/bin/env python3
"""Gravity evaluation micro-benchmark: Evrard -n N after one full step, then K evaluations of the Barnes-Hut
traversal on the same tree and multipoles (interaction lists + P2P + M2P + combine + spill), timed with device events.
Run under rocprofv3 --kernel-trace --stats for the per-kernel split. usage: grav_micro.py [-n 200] [-k 5]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from sphexa_amd.app.simulation import Simulation  # noqa: E402
from sphexa_amd.ops import gravity as G  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-n", type=int, default=200)
    ap.add_argument("-k", type=int, default=5)
    a = ap.parse_args()
    sim = Simulation("evrard", n=a.n)
    sim.step()
    d, dom = sim.d, sim.domain
    mh = sim.propagator.gravity
    mh.upsweep(d, dom)
    s, e = dom.start_index(), dom.end_index()
    acc = [torch.zeros(d.size, dtype=torch.float32, device=d.device) for _ in range(3)]
    args = (dom.octree, mh.centers, mh.multipoles, s, e, d["x"], d["y"], d["z"], d["h"], d["m"], d.g, *acc)
    G.compute_gravity(*args)  # warm
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st = {}
    t0.record()
    for _ in range(a.k):
        G.compute_gravity(*args, stats=st, defer=True)
    t1.record()
    torch.cuda.synchronize()
    ms = t0.elapsed_time(t1) / a.k
    print(f"variant {os.environ.get('SPHX_HIP_VARIANT', 'default')}: evrard -n {a.n} ({e - s} particles) gravity "
          f"evaluation {ms:.3f} ms")
    # consistency: two more evaluations with statistics (identical inputs: identical results)
    res = []
    for _ in range(2):
        acc2 = [torch.zeros_like(v) for v in acc]
        st = {}
        eg = G.compute_gravity(*args[:-3], *acc2, stats=st)
        res.append((acc2, eg, st))
    (a0, e0, s0), (a1, e1, s1) = res
    same = all(torch.equal(u, v) for u, v in zip(a0, a1))
    print(f"  stats {s0}\n  egrav {e0:.9e} / {e1:.9e}, repeat identical: {same}, "
          f"|a| max {float(torch.sqrt(a0[0]**2 + a0[1]**2 + a0[2]**2).max()):.6e}")


if __name__ == "__main__":
    main()
