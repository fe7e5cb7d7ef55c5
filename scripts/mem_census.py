#!/usr/bin/env python3
"""Census of the device memory a test case holds between steps: particle fields, neighbor lists, record workspaces,
tree and scratch, in bytes per particle (memory item of the round-2 plan).

  python scripts/mem_census.py --init sedov -n 200 --steps 2
"""

import argparse
import gc
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--init", default="sedov")
    ap.add_argument("-n", type=int, default=200)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--at-sync", action="store_true", help="census at the start of the last step's domain sync "
                    "(after the record workspaces are released) and the sync's own peak")
    args = ap.parse_args()
    from sphexa_amd.app.simulation import Simulation
    from sphexa_amd.parallel.comm import init_distributed

    comm = init_distributed("nccl")
    sim = Simulation(args.init, n=args.n, prop="ve", device=torch.device("cuda", 0), comm=comm, out=None, quiet=True)
    for _ in range(args.steps - (1 if args.at_sync else 0)):
        sim.step()
    torch.cuda.synchronize()
    if args.at_sync:
        dom_cls = type(sim.domain)
        orig = dom_cls.sync

        def sync(self, *a, **k):
            torch.cuda.synchronize()
            census(sim, args, "at sync start")
            torch.cuda.reset_peak_memory_stats()
            base = torch.cuda.memory_allocated()
            r = orig(self, *a, **k)
            torch.cuda.synchronize()
            n = sim.d.numParticlesGlobal
            print(f"sync: allocated at start {base / n:.0f} B/p, peak inside {torch.cuda.max_memory_allocated() / n:.0f}"
                  f" B/p, at end {torch.cuda.memory_allocated() / n:.0f} B/p")
            return r

        dom_cls.sync = sync
        sim.step()
        return
    census(sim, args, "between steps")


def census(sim, args, where):
    n = sim.d.numParticlesGlobal
    d = sim.d
    names = {}
    for f, t in d._buf.items():
        if isinstance(t, torch.Tensor) and t.is_cuda:
            names[t.untyped_storage().data_ptr()] = f"field {f} ({'active' if d._state.get(f) else 'released'})"
    for attr, v in vars(d).items():
        if isinstance(v, torch.Tensor) and v.is_cuda:
            names.setdefault(v.untyped_storage().data_ptr(), f"d.{attr}")
    nl = getattr(sim.propagator, "nl", None)
    if nl is not None and nl.nidx is not None and nl.nidx.is_cuda:
        names[nl.nidx.untyped_storage().data_ptr()] = "neighbor lists"
    seen = {}
    for o in gc.get_objects():
        try:
            if isinstance(o, torch.Tensor) and o.is_cuda:
                st = o.untyped_storage()
                seen[st.data_ptr()] = (st.nbytes(), tuple(o.shape), o.dtype)
        except Exception:
            pass
    total = sum(v[0] for v in seen.values())
    print(f"[{where}] {args.init} -n {args.n}: {n} particles; live tensors {total / 2**30:.2f} GiB ({total / n:.0f} B/particle); "
          f"allocator: allocated {torch.cuda.memory_allocated() / 2**30:.2f} GiB, peak "
          f"{torch.cuda.max_memory_allocated() / 2**30:.2f} GiB ({torch.cuda.max_memory_allocated() / n:.0f} B/particle)")
    rows = sorted(seen.items(), key=lambda kv: -kv[1][0])
    for ptr, (nb, shape, dt) in rows[:12]:
        print(f"{nb / n:8.1f} B/p  {nb / 2**20:10.1f} MiB  {str(dt):14s} {str(shape):22s} {names.get(ptr, '')}")


if __name__ == "__main__":
    main()
