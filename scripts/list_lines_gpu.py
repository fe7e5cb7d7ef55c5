#!/usr/bin/env python3
"""distinct 128-B lines per lane-parallel gather step of the GPU neighbor lists of a short run (16-B records), and the
list order of one group's first lanes; SPHX_SORT_LISTS selects the list order (csrc/hip/neighbors.hip)

usage: python scripts/list_lines_gpu.py [case=sedov] [n=64]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from sphexa_amd.app.simulation import Simulation
    from sphexa_amd.ops.neighbors import decode_packed

    case = sys.argv[1] if len(sys.argv) > 1 else "sedov"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    sim = Simulation(case, n=n, device=torch.device("cuda", 0), quiet=True)
    sim.run(2)
    torch.cuda.synchronize()
    idx, valid = decode_packed(sim.propagator.nl)
    G = idx.shape[0] // 64
    idx = idx[:G * 64].view(G, 64, -1)
    valid = valid[:G * 64].view(G, 64, -1)
    tot = steps = 0
    for g in range(0, G, max(G // 400, 1)):
        lines = torch.where(valid[g], idx[g] * 16 // 128, -1)
        for k in range(lines.shape[1]):
            col = lines[:, k]
            col = col[col >= 0]
            if col.numel():
                tot += int(torch.unique(col).numel())
                steps += 1
    print(f"SPHX_SORT_LISTS={os.environ.get('SPHX_SORT_LISTS', '0')} {case} -n {n}: {tot / steps:.2f} lines per step "
          f"({steps} steps), sets checksum {int(torch.where(valid, idx, 0).sum())}")
    g = G // 2
    print("group", g, "lane 0..2 first 12 entries:", idx[g, :3, :12].tolist())


if __name__ == "__main__":
    main()
