#!/usr/bin/env python3
"""Host-side (Python) profile of the time step at a launch-bound size: cProfile over K steps after W warmup steps,
top functions by own time. usage: python scripts/host_profile.py [--init evrard] [-n 100] [--steps 20]"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--init", default="evrard")
    ap.add_argument("-n", type=int, default=100)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--top", type=int, default=45)
    ap.add_argument("--sort", default="tottime")
    ap.add_argument("--filter", default=None, help="regex on file:line(function) of the printed rows")
    args = ap.parse_args()
    from sphexa_amd.app.simulation import Simulation

    sim = Simulation(args.init, n=args.n, device=torch.device("cuda", 0), out=None, quiet=True)
    sim.propagator.timer.sync = False  # as bench.py: no device synchronization at the substep boundaries
    sim.propagator.defer_host = True  # as bench.py
    for _ in range(args.warmup):
        sim.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sim.step()
    torch.cuda.synchronize()
    plain = (time.perf_counter() - t0) / args.steps
    prof = cProfile.Profile()
    prof.enable()
    for _ in range(args.steps):
        sim.step()
    torch.cuda.synchronize()
    prof.disable()
    s = io.StringIO()
    st = pstats.Stats(prof, stream=s)
    st.sort_stats(args.sort)
    if args.filter:
        st.print_stats(args.filter, args.top)
    else:
        st.print_stats(args.top)
    print(f"{args.init} -n {args.n}: {1e3 * plain:.3f} ms/step without the profiler")
    print(s.getvalue())


if __name__ == "__main__":
    main()
