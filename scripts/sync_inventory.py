#!/usr/bin/env python3
"""Inventory of the host synchronizations of one time step (torch sync-debug mode): which lines of the package copy
device values to the host, per step.

  python scripts/sync_inventory.py [--init evrard] [-n 50]              one rank
  python scripts/sync_inventory.py --ranks 2 [--init evrard] [-n 50]    N ranks sharing cuda:0 over gloo
  ... --defer                                                           the bench.py / sphexa CLI configuration:
                                                                        time-step packet and conserved quantities
                                                                        collected one step late (Propagator.defer_host)

Event waits (torch.cuda.Event.synchronize on events recorded earlier in the step or the step before: pinned copies
collected once the stream is known to be past them) are not sync-debug warnings; they are counted separately
("event waits").

With several ranks the gloo staging copies of parallel/comm.py (host bounce buffers of a backend that RCCL replaces)
are reported separately and not counted: the count is what an RCCL run synchronizes.
"""
import argparse
import collections
import json
import os
import sys
import traceback
import warnings

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

STAGING = ("_stage_host", "_stage_dev")  # parallel/comm.py gloo bounce-buffer copies


def inventory(init: str, n: int, steps_before: int = 2, comm=None, steps: int = 1, defer: bool = False,
              events: list | None = None):
    """(counted sites, staging sites) of one step after ``steps_before`` steps (``steps`` > 1: lists of them, one per
    step: steps in which a per-step octree is rebalanced add the synchronous rebalance loop, octree.update_tree)"""
    from sphexa_amd.app.simulation import Simulation

    sim = Simulation(init, n=n, prop="ve", device=torch.device("cuda", 0), comm=comm, out=None, quiet=True)
    sim.propagator.defer_host = defer
    sim.run(steps_before)
    ev_count = [0]
    ev_sync = torch.cuda.Event.synchronize

    def counted_sync(self):
        ev_count[0] += 1
        return ev_sync(self)
    per_step = []
    sites, staged = collections.Counter(), collections.Counter()

    def hook(message, category, filename, lineno, file=None, line=None):
        frames = [fr for fr in traceback.extract_stack()[:-1] if "sphexa_amd" in fr.filename]
        if not frames:
            return
        if frames[-1].name in STAGING:
            fr = frames[-2] if len(frames) > 1 else frames[-1]
            staged[f"{os.path.relpath(fr.filename)}:{fr.lineno}"] += 1
            return
        fr = frames[-1]
        sites[f"{os.path.relpath(fr.filename)}:{fr.lineno} {fr.line}"] += 1

    warnings.showwarning = hook
    warnings.simplefilter("always")
    for _ in range(steps):
        sites.clear()
        staged.clear()
        ev_count[0] = 0
        torch.cuda.Event.synchronize = counted_sync
        torch.cuda.set_sync_debug_mode("warn")
        try:
            sim.run(1)
        finally:
            torch.cuda.set_sync_debug_mode("default")
            torch.cuda.Event.synchronize = ev_sync
        if events is not None:
            events.append(ev_count[0])
        per_step.append((collections.Counter(sites), collections.Counter(staged)))
    if steps == 1:
        return per_step[0]
    return [p[0] for p in per_step], [p[1] for p in per_step]


def _worker(rank, size, port, init, n, q, steps=1, defer=False):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(size))
    dist.init_process_group("gloo", rank=rank, world_size=size)
    from sphexa_amd.parallel.comm import Comm

    events = []
    sites, staged = inventory(init, n, comm=Comm(), steps=steps, defer=defer, events=events)
    if steps == 1:
        q.put((rank, dict(sites), dict(staged), events))
    else:
        q.put((rank, [dict(x) for x in sites], [dict(x) for x in staged], events))
    dist.barrier()
    dist.destroy_process_group()


def multi_rank(size: int, init: str, n: int, steps: int = 1, defer: bool = False):
    """per rank (rank, sites, staging sites, event waits per step)"""
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, size, port, init, n, q, steps, defer)) for r in range(size)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=600) for _ in procs)
    for p in procs:
        p.join(timeout=120)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--init", default="evrard")
    ap.add_argument("-n", type=int, default=50)
    ap.add_argument("--ranks", type=int, default=1)
    ap.add_argument("--json", action="store_true")
    ap.add_argument("--defer", action="store_true", help="host values collected one step late (bench.py / CLI)")
    args = ap.parse_args()
    if args.ranks == 1:
        events = []
        results = [(0,) + inventory(args.init, args.n, defer=args.defer, events=events) + (events,)]
    else:
        results = multi_rank(args.ranks, args.init, args.n, defer=args.defer)
    for rank, sites, staged, events in results:
        sites, staged = collections.Counter(sites), collections.Counter(staged)
        if args.json:
            print(json.dumps({"rank": rank, "syncs": sum(sites.values()), "staging": sum(staged.values()),
                              "event_waits": sum(events), "sites": dict(sites)}))
            continue
        print(f"rank {rank}: {sum(sites.values())} synchronizing calls in one step ({args.init} -n {args.n}, "
              f"{args.ranks} ranks{', deferred host values' if args.defer else ''}; + {sum(staged.values())} gloo "
              f"staging copies not counted; {sum(events)} event waits):")
        for k, v in sites.most_common():
            print(f"{v:4d}  {k}")


if __name__ == "__main__":
    main()
