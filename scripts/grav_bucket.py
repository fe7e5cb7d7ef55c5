#!/usr/bin/env python3
"""What-if for the gravity tree's leaf size (verdict r2 item 3b: fewer P2P pairs per target): the same Evrard particles
(sorted, after the first domain sync) get octrees with leaves of at most 64 (production, shared with the neighbor
search), 32, 16 and 8 particles; for each the upsweep and the evaluation (list + M2P + P2P) are timed and P2P / M2P per
target and the deviation of the accelerations from the bucket-64 result are printed.
usage: python scripts/grav_bucket.py [-n 200] [--buckets 64,32,16,8]"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-n", type=int, default=200)
    ap.add_argument("--buckets", default="64,32,16,8")
    args = ap.parse_args()
    from sphexa_amd.app.simulation import Simulation
    from sphexa_amd.ops import gravity as G
    from sphexa_amd.ops import octree as O

    dev = torch.device("cuda", 0)
    sim = Simulation("evrard", n=args.n, device=dev, out=None, quiet=True)
    d, dom = sim.d, sim.domain
    n = d.size
    x, y, z, h, m, keys = (d[f][:n] for f in ("x", "y", "z", "h", "m", "keys"))
    ref = None
    for b in (int(v) for v in args.buckets.split(",")):
        tree, counts = O.update_tree(None, keys, b)
        ot = O.build_octree(tree, counts, keys, x, y, z, 0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            c, mp = G.upsweep(ot, x, y, z, m, dom.box, dom.theta)
        torch.cuda.synchronize()
        tu = (time.perf_counter() - t0) / 3
        ax, ay, az = (torch.zeros(n, dtype=torch.float32, device=dev) for _ in range(3))
        st = {}
        times = []
        for it in range(4):
            ax.zero_(), ay.zero_(), az.zero_()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            G.compute_gravity(ot, c, mp, 0, n, x, y, z, h, m, 1.0, ax, ay, az, stats=st)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
        a = torch.stack([ax, ay, az]).double()
        if ref is None:
            ref = a
        amag = ref.norm(dim=0)
        err = ((a - ref).norm(dim=0) / amag).float()
        q = torch.quantile(err[:: max(1, n // 1_000_000)], torch.tensor([0.5, 0.99], device=dev)).tolist()
        print(f"bucket {b}: leaves {ot.num_leaves} nodes {ot.num_nodes} upsweep {1e3 * tu:.2f} ms, evaluation "
              f"{1e3 * min(times[1:]):.2f} ms, P2P/target {st['p2p'] / n:.0f} M2P/target {st['m2p'] / n:.0f} "
              f"max P2P {st['max_p2p']} | deviation from bucket 64: p50 {q[0]:.2e} p99 {q[1]:.2e} "
              f"max {err.max().item():.2e}", flush=True)


if __name__ == "__main__":
    main()
