#!/usr/bin/env python3
"""Headline benchmark: particle-updates/s of the VE-SPH Sedov blast, ``--init sedov -n 400`` (64 M particles).

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N > 1 the driver starts one process per
GPU with torch.distributed.run. W untimed steps, then exactly K timed steps bracketed by barrier + device sync,
max over ranks, rank 0 prints one JSON line. The whole time step is inside the timed region: domain sync (SFC keys,
sort, octree, halo discovery), neighbor search with h iteration, the five VE loops, EOS, four halo exchanges,
global dt reduction and the position/energy/h update.

Scaling: the problem (64 M particles) is fixed as N grows -> strong scaling.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

BASELINE_VALUE = None  # the reference publishes no throughput numbers


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("-n", type=int, default=400, help="particles per dimension (n^3 total)")
    ap.add_argument("--prop", default="ve")
    ap.add_argument("--verbose", action="store_true")
    args = ap.parse_args()

    from sphexa_amd.models import particles as P
    from sphexa_amd.models.init.sedov import SedovGrid
    from sphexa_amd.models.propagators import propagator_factory
    from sphexa_amd.parallel.comm import init_distributed
    from sphexa_amd.parallel.domain import Domain

    comm = init_distributed("nccl" if torch.cuda.is_available() else "gloo")
    rank, size = comm.rank, comm.size
    if torch.cuda.is_available():
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")

    d = P.ParticlesData(device)
    prop = propagator_factory(args.prop, False, sys.stdout if (args.verbose and rank == 0) else None, rank, True)
    prop.activate_fields(d)
    prop.timer.sync = args.verbose
    init = SedovGrid()
    box = init.init(rank, size, args.n, d)
    bucket = max(64, d.numParticlesGlobal // (100 * size))
    domain = Domain(comm, box, bucket_size_focus=64, bucket_size=bucket)
    prop.sync(domain, d)

    def step():
        prop.step(domain, d)
        d.iteration += 1

    for _ in range(args.warmup):
        step()

    comm.barrier()
    if device.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    comm.barrier()
    if device.type == "cuda":
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0

    dt = comm.allreduce_scalar(dt, "max", device=device)
    ms = 1000.0 * dt / max(args.steps, 1)
    value = d.numParticlesGlobal * args.steps / dt
    if rank == 0:
        out = {
            "metric": "particle-updates/sec (whole node), Sedov -n 400",
            "value": value,
            "unit": "particle-updates/s",
            "n_gpus": size,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": (value / BASELINE_VALUE) if BASELINE_VALUE else None,
            "dtype": "fp64 coordinates + fp32 hydro (reference precision mix)",
            "data": "synthetic (built-in Sedov lattice initial conditions)",
            "config": {"model": f"sedov-ve -n {args.n} ({d.numParticlesGlobal} particles)",
                       "global_batch": d.numParticlesGlobal, "seq_len": 1,
                       "parallelism": f"sfc-domain-decomposition x{size}"},
        }
        print(json.dumps(out), flush=True)
        if args.verbose:
            nsteps = max(prop.timer.num_accum, 1)
            for k, v in prop.timer.accum.items():
                print(f"# substep {k:28s} {1000.0 * v / nsteps:10.3f} ms/step", file=sys.stderr)
            if device.type == "cuda":
                print(f"# max memory allocated {torch.cuda.max_memory_allocated() / 2**30:.2f} GiB", file=sys.stderr)


if __name__ == "__main__":
    main()
