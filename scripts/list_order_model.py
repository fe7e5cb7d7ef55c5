#!/usr/bin/env python3
"""Distinct 128-B lines per wave gather instruction of the SPH pair loops, modelled on a Morton-ordered lattice, for
different orders of each lane's neighbor list (the texture addresser pays ~2 cycles per distinct line per instruction,
profiles/r5/gather_ta_micro.md). 64 consecutive particles form a group (one wave); at step k every lane gathers its
k-th neighbor's record of REC bytes. Output: mean lines per step for each order.

usage: python scripts/list_order_model.py [n=48] [groups=150] [radius=2.9]
"""
import sys

import numpy as np
from scipy.spatial import cKDTree


def spread(v):
    v = v.astype(np.uint64)
    r = np.zeros_like(v)
    for b in range(21):
        r |= ((v >> np.uint64(b)) & np.uint64(1)) << np.uint64(3 * b)
    return r


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 48
    ngroups = int(sys.argv[2]) if len(sys.argv) > 2 else 150
    radius = float(sys.argv[3]) if len(sys.argv) > 3 else 2.9
    g = np.arange(n)
    X, Y, Z = np.meshgrid(g, g, g, indexing="ij")
    P = np.stack([X.ravel(), Y.ravel(), Z.ravel()], 1).astype(np.int64)
    key = (spread(P[:, 0]) << np.uint64(2)) | (spread(P[:, 1]) << np.uint64(1)) | spread(P[:, 2])
    P = P[np.argsort(key, kind="stable")]
    tree = cKDTree(P.astype(float), boxsize=n)
    groups = np.random.default_rng(0).choice(len(P) // 64, ngroups, replace=False)
    nbrs = {}
    for gi in groups:
        for i in range(gi * 64, gi * 64 + 64):
            nb = np.array(sorted(tree.query_ball_point(P[i].astype(float), radius)))
            nbrs[i] = nb[nb != i]

    def lines(order, rec):
        tot = steps = 0
        for gi in groups:
            lists = []
            for i in range(gi * 64, gi * 64 + 64):
                nb = nbrs[i]
                lists.append(nb[np.lexsort((nb, order(nb, i)))])
            for k in range(max(len(l) for l in lists)):
                tot += len({(l[k] * rec) // 128 for l in lists if k < len(l)})
                steps += 1
        return tot / steps

    orders = {
        "source index (search order today)": lambda nb, i: np.zeros(len(nb)),
        "source x, then index": lambda nb, i: P[nb][:, 0],
        "source (x, y), then index": lambda nb, i: P[nb][:, 0] * 100000 + P[nb][:, 1],
        "offset octant, then index": lambda nb, i: ((P[nb] - P[i]) > 0) @ np.array([4, 2, 1]),
    }
    print(f"lattice {n}^3, {ngroups} groups of 64, radius {radius} spacings")
    for rec in (16, 32):
        for name, f in orders.items():
            print(f"{rec:3d}-B records  {name:36s} {lines(f, rec):6.2f} lines per gather")


if __name__ == "__main__":
    main()
