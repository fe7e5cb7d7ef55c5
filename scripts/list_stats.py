#!/usr/bin/env python3
"""Statistics of the packed GPU neighbor lists of a test case (memory item of the round-2 plan).

Reports list rows per group and bytes per particle of the packed lists, the jump-slot share and the int32 layout it
replaced (ngmax stride). The design numbers of packed_list.hpp (share of list steps that fit 15 bits) came from the
int32 lists of the same cases: profiles/r2_list_stats.md.

  python scripts/list_stats.py --init sedov -n 400
"""

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--init", default="sedov")
    ap.add_argument("-n", type=int, default=400)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--sample-groups", type=int, default=4096)
    args = ap.parse_args()
    from sphexa_amd.app.simulation import Simulation
    from sphexa_amd.ops.neighbors import (GROUP, NeighborList, decode_packed, packed_table_ints,
                                          packed_table_region)
    from sphexa_amd.parallel.comm import init_distributed

    comm = init_distributed("nccl")
    sim = Simulation(args.init, n=args.n, prop="ve", device=torch.device("cuda", 0), comm=comm, out=None, quiet=True)
    from sphexa_amd.ops.neighbors import packed_table_ints as _pti
    for k in range(args.steps):
        sim.step()
        q = sim.propagator.nl
        if q is not None and q.grouped:
            Gq = (q.last - q.first + GROUP - 1) // GROUP
            nrq = q.nidx[:Gq * _pti(q.ngmax)].view(Gq, -1)[:, 0].float()
            print(f"step {k}: rows used {q.rows_used}, plan {q.plan}, pool {q.nidx.numel() * 4 / (q.last - q.first):.0f} "
                  f"B/p, rows/group mean {float(nrq.mean()):.2f} max {int(nrq.max())}, rounds {sim.d.nc_rounds:.2f}",
                  flush=True)
            dom = sim.domain if hasattr(sim, "domain") else None
            kk = sim.d["keys"][q.first:q.last]
            print(f"   keys sorted {bool((kk[1:] >= kk[:-1]).all())}, unique {int(torch.unique(kk).numel())}, "
                  f"box lo {getattr(dom, 'box', None) and list(dom.box.lo)} hi {getattr(dom, 'box', None) and list(dom.box.hi)}, "
                  f"leaves {getattr(dom, 'octree', None) and dom.octree.num_leaves}", flush=True)
    nl, d = sim.propagator.nl, sim.d
    n = nl.last - nl.first
    G = (n + GROUP - 1) // GROUP
    cap = (nl.nidx.numel() - packed_table_region(G, nl.ngmax)) // 256
    nc = d["nc"][nl.first:nl.last].to(torch.int64) - 1
    print(f"case {args.init} -n {args.n}: {n} particles, {G} groups, ngmax {nl.ngmax}, mean list {float(nc.float().mean()):.1f}")
    print(f"rows used {nl.rows_used} ({nl.rows_used / G:.2f} per group), pool {cap} rows; "
          f"packed lists {nl.nidx.numel() * 4 / n:.0f} B/particle (used rows {nl.rows_used * 1024 / n:.0f}), "
          f"int32 at the ngmax stride {4 * ((nl.ngmax + 3) // 4 * 4):.0f} B/particle")
    Ti = packed_table_ints(nl.ngmax)
    tab = nl.nidx[:G * Ti].view(G, Ti)
    nrows = tab[:, 0].to(torch.int64)
    alloc = (tab[:, 1:] != 0).sum(dim=1)  # rows named by the table (row 0 aside): allocated incl. earlier h rounds
    print(f"rows per group (final round): mean {float(nrows.float().mean()):.2f}, histogram from "
          f"{int(nrows.min())}: {torch.bincount(nrows - nrows.min()).tolist()}")
    print(f"rows allocated per group (incl. earlier h-iteration rounds): mean {float(alloc.float().mean()):.2f}, "
          f"histogram from {int(alloc.min())}: {torch.bincount(alloc - alloc.min()).tolist()}")
    print(f"h-iteration rounds per group (last search): {getattr(d, 'nc_rounds', float('nan'))}")
    # entries per slot (jump and padding slots) in a sample of groups: their tables + the whole row pool
    k = min(args.sample_groups, G)
    buf = torch.cat([nl.nidx[:k * Ti].cpu(), torch.zeros(packed_table_region(k, nl.ngmax) - k * Ti, dtype=torch.int32),
                     nl.nidx[packed_table_region(G, nl.ngmax):].cpu()])
    last = min(nl.first + k * GROUP, nl.last)
    idx, valid = decode_packed(NeighborList(buf, nl.first, last, nl.ngmax, True))
    ent = int(valid.sum())
    slots = int(buf[:k * Ti].view(k, Ti)[:, 0].sum()) * 8 * GROUP
    print(f"sample {k} groups: entries {ent} (capped nc sum {int(nc[:last - nl.first].clamp(max=nl.ngmax).sum())}), "
          f"{slots} slots in their rows: {ent / max(slots, 1):.3f} entries per slot")


if __name__ == "__main__":
    main()
