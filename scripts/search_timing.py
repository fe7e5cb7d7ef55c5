#!/usr/bin/env python3
"""Time the GPU neighbor search alone (on the initial conditions of a test case), e.g. to A/B search variants:
  SPHX_HIP_VARIANT=<tag> python scripts/search_timing.py --init sedov -n 400"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--init", default="sedov")
    ap.add_argument("-n", type=int, default=400)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--presteps", type=int, default=0, help="time steps run first (converged h, steady-state lists)")
    ap.add_argument("--no-iterate", action="store_true", help="one round, no h iteration (timing variants whose lists "
                    "are unusable would otherwise repeat rounds)")
    args = ap.parse_args()
    from sphexa_amd.app.simulation import Simulation
    from sphexa_amd.ops import neighbors as N
    from sphexa_amd.parallel.comm import init_distributed

    comm = init_distributed("nccl")
    sim = Simulation(args.init, n=args.n, prop="ve", device=torch.device("cuda", 0), comm=comm, out=None, quiet=True)
    for _ in range(args.presteps):
        sim.step()
    dom, d, prop = sim.domain, sim.d, sim.propagator  # (variants may leave lists unusable: only the search runs now)
    N.ALLOW_NC_FAIL = True
    ts = []
    for _ in range(args.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        # (iterate_h: the production kernel; after the first call h is converged and the search is one round)
        N.find_neighbors(d, dom.octree, dom.box, dom.start_index(), dom.end_index(), iterate_h=not args.no_iterate)
        torch.cuda.synchronize()
        ts.append(1e3 * (time.perf_counter() - t0))
    print(f"search {os.environ.get('SPHX_HIP_VARIANT', 'default')}: " + " ".join(f"{t:.1f}" for t in ts) + " ms",
          flush=True)
    if N.COLLECT_STATS:
        print(f"per group: rounds {d.nc_rounds:.2f} touched leaves {d.nc_leaves:.1f} staged candidates "
              f"{d.nc_staged:.0f} hits {d.nc_hits:.0f} ({d.nc_hits / max(d.nc_staged, 1) / 64:.3f} per lane and "
              f"candidate) inside 8 sub-group boxes {d.nc_subbox:.0f}", flush=True)


if __name__ == "__main__":
    main()
