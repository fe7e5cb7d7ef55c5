#!/usr/bin/env python3
"""Per-group source unions of the packed GPU neighbor lists (design data of the LDS-staged pair loops).

For a sample of 64-target groups: the chunk-table size nch, the list blocks nblk, the exact union of the group's
neighbor indices (plus its own 64 targets), the union of per-chunk offset ranges [min, max] and the full chunk count
x 64 -- i.e. how many source records a group would have to hold in LDS for each way of staging them.

  python scripts/union_stats.py --init sedov -n 100
"""

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def pct(t: torch.Tensor, qs=(0.5, 0.9, 0.99, 1.0)):
    t = t.float()
    return " ".join(f"p{int(q * 100)} {float(torch.quantile(t, q)):.0f}" for q in qs) + f" mean {float(t.mean()):.1f}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--init", default="sedov")
    ap.add_argument("-n", type=int, default=100)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--sample-groups", type=int, default=8192)
    args = ap.parse_args()
    from sphexa_amd.app.simulation import Simulation
    from sphexa_amd.ops.neighbors import GROUP, NeighborList, decode_packed, packed_table_ints, packed_table_region
    from sphexa_amd.parallel.comm import init_distributed

    comm = init_distributed("nccl")
    sim = Simulation(args.init, n=args.n, prop="ve", device=torch.device("cuda", 0), comm=comm, out=None, quiet=True)
    for _ in range(args.steps):
        sim.step()
    nl = sim.propagator.nl
    n = nl.last - nl.first
    G = (n + GROUP - 1) // GROUP
    Ti = packed_table_ints(nl.ngmax)
    k = min(args.sample_groups, G)
    g0 = (G - k) // 2  # a sample from the middle of the range
    tab_all = nl.nidx[:G * Ti].view(G, Ti)
    tab = tab_all[g0:g0 + k].cpu()
    buf = torch.cat([tab.reshape(-1), torch.zeros(packed_table_region(k, nl.ngmax) - k * Ti, dtype=torch.int32),
                     nl.nidx[packed_table_region(G, nl.ngmax):].cpu()])
    first = nl.first + g0 * GROUP
    last = min(first + k * GROUP, nl.last)
    idx, valid = decode_packed(NeighborList(buf, first, last, nl.ngmax, True))
    kk = (last - first) // GROUP  # whole groups only
    last = first + kk * GROUP
    tab = tab[:kk]
    S = idx.shape[1]
    idx = idx[:kk * GROUP].view(kk, GROUP * S)
    valid = valid[:kk * GROUP].view(kk, GROUP * S)
    own = (first + torch.arange(kk * GROUP)).view(kk, GROUP)
    big = torch.iinfo(torch.int64).max
    allidx = torch.cat([torch.where(valid, idx, big), own], dim=1)
    srt, _ = allidx.sort(dim=1)
    newv = torch.ones_like(srt, dtype=torch.bool)
    newv[:, 1:] = srt[:, 1:] != srt[:, :-1]
    newv &= srt != big
    uexact = newv.sum(dim=1)
    # per-chunk offset ranges: chunk id = j >> 6 in aligned terms is not the search's chunk; use the table's chunks:
    nch = (tab[:kk, 1] & 0x3FF).long()
    nblk = tab[:kk, 0].long()
    # range union by 64-aligned blocks of the source index (an upper bound proxy of per-chunk ranges)
    blk = torch.where(srt != big, srt >> 6, -1)
    off = srt & 63
    # min/max offset per (group, block): positions where a block starts/ends in the sorted row
    start = torch.ones_like(srt, dtype=torch.bool)
    start[:, 1:] = blk[:, 1:] != blk[:, :-1]
    end = torch.ones_like(srt, dtype=torch.bool)
    end[:, :-1] = blk[:, :-1] != blk[:, 1:]
    live = blk >= 0
    lo = torch.where(start & live, off, 0).sum(dim=1)
    hi = torch.where(end & live, off + 1, 0).sum(dim=1)
    urange = hi - lo
    nblocks = (start & live).sum(dim=1)
    nc = sim.d["nc"][first:last].long().cpu() - 1
    print(f"case {args.init} -n {args.n}: {n} particles, {G} groups, sample {kk} groups; mean nc {float(nc.float().mean()):.1f}")
    print(f"  nch (chunk-table slots)         {pct(nch)}")
    print(f"  nblk (list blocks)              {pct(nblk)}  -> lane steps {8 * float(nblk.float().mean()):.1f}")
    print(f"  exact union (+ own 64)          {pct(uexact)}")
    print(f"  64-aligned blocks touched       {pct(nblocks)}")
    print(f"  union of per-block [min,max]    {pct(urange)}")
    print(f"  full chunks nch * 64            {pct(nch * 64)}")
    print(f"  pair uses per union record      {float((valid.sum(dim=1)).float().mean() / uexact.float().mean()):.2f}")


if __name__ == "__main__":
    main()
