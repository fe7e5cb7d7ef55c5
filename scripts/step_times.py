#!/usr/bin/env python3
"""Per-step wall times of the bench configuration (defer_host as in bench.py), each step bracketed by a device
synchronization, plus the caching allocator's device malloc/free counts per step: locates steps that cost more than
the kernel sum of a trace (host syncs, allocator calls, a heavier step type).
  python scripts/step_times.py --init sedov -n 400 --warmup 3 --steps 10 [--nosync]"""
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
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--ptrs", action="store_true", help="print the field buffers' device addresses per synced step")
    args = ap.parse_args()
    from sphexa_amd.app.simulation import Simulation
    from sphexa_amd.parallel.comm import init_distributed

    comm = init_distributed("nccl")
    dev = torch.device("cuda", 0)
    sim = Simulation(args.init, n=args.n, prop="ve", device=dev, comm=comm, out=None, quiet=True)
    sim.propagator.defer_host = True
    for _ in range(args.warmup):
        sim.step()
    torch.cuda.synchronize()

    def counts():
        s = torch.cuda.memory_stats()
        return s.get("num_device_alloc", 0), s.get("num_device_free", 0), s.get("num_alloc_retries", 0)

    c0 = counts()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sim.step()
    torch.cuda.synchronize()
    block = 1e3 * (time.perf_counter() - t0) / args.steps
    c1 = counts()
    print(f"block of {args.steps} steps: {block:.2f} ms/step; device allocs/frees/retries "
          f"{c1[0] - c0[0]}/{c1[1] - c0[1]}/{c1[2] - c0[2]}", flush=True)
    ts = []
    for k in range(args.steps):
        a = counts()
        t = time.perf_counter()
        sim.step()
        torch.cuda.synchronize()
        ts.append(1e3 * (time.perf_counter() - t))
        b = counts()
        print(f"step {k}: {ts[-1]:.2f} ms  allocs/frees {b[0] - a[0]}/{b[1] - a[1]}", flush=True)
        if args.ptrs:
            d = sim.d
            bufs = {n: t.data_ptr() for n, t in d._buf.items()}
            nl = sim.propagator.nl
            for attr in ("nidx", "rec", "tab"):
                t = getattr(nl, attr, None)
                if torch.is_tensor(t):
                    bufs["nl." + attr] = t.data_ptr()
            print("  ptrs " + " ".join(f"{n}={v >> 20:x}" for n, v in sorted(bufs.items())), flush=True)
    print(f"synced steps: mean {sum(ts) / len(ts):.2f} min {min(ts):.2f} max {max(ts):.2f} ms", flush=True)


if __name__ == "__main__":
    main()
