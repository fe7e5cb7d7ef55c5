#!/usr/bin/env python3
"""What-if for gravity target groups smaller than a wave (verdict r2 item 3b): the GPU traversal takes groups of 64
consecutive targets; groups of 32 (16) are emulated by evaluating a target array in which each group's first 32 (16)
particles are repeated to fill the wave, so the group box is that of 32 (16) targets. Prints P2P / M2P per unique
target and the evaluation time per unique target set (Evrard ICs; same tree and multipoles).
usage: python scripts/grav_group_size.py [-n 200]"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-n", type=int, default=200)
    args = ap.parse_args()
    from sphexa_amd.app.simulation import Simulation
    from sphexa_amd.ops import gravity as G

    dev = torch.device("cuda", 0)
    sim = Simulation("evrard", n=args.n, device=dev, out=None, quiet=True)
    d, dom = sim.d, sim.domain
    n = dom.end_index() - dom.start_index()
    ot = dom.octree
    c, mp = G.upsweep(ot, d["x"], d["y"], d["z"], d["m"], dom.box, dom.theta)
    base = {f: d[f][:d.size] for f in ("x", "y", "z", "h", "m")}
    for sub in (64, 32, 16):
        rep = 64 // sub
        ng = (n + 63) // 64
        idx = torch.arange(ng * 64, device=dev).clamp(max=n - 1).view(ng, 64)
        # each 64-group -> rep groups of `sub` targets, each repeated rep times to fill the wave
        lay = idx.view(ng, rep, sub).repeat_interleave(rep, dim=2).reshape(-1)
        T = lay.numel()
        arr = {f: torch.cat([base[f], base[f][lay]]) for f in base}
        ax, ay, az = (torch.zeros(d.size + T, dtype=torch.float32, device=dev) for _ in range(3))
        st = {}
        for it in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            G.compute_gravity(ot, c, mp, d.size, d.size + T, arr["x"], arr["y"], arr["z"], arr["h"], arr["m"], 1.0,
                              ax, ay, az, stats=st)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
        print(f"groups of {sub}: P2P/target {st['p2p'] / T:.0f} M2P/target {st['m2p'] / T:.0f} max P2P {st['max_p2p']} "
              f"time per unique target set {1e3 * dt / rep:.2f} ms (evaluated {T} targets in {1e3 * dt:.2f} ms)",
              flush=True)


if __name__ == "__main__":
    main()
