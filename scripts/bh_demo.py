"""Single-GPU Barnes-Hut demo (reference ryoanji/test/demo.cu:48-107): 2^power - 1 random cube bodies (extent 3,
h from 100 neighbors), theta 0.6, ncrit (bucket) 64, order-P multipole far field; times the traversal of the
order-P path and of the production quadrupole path, then checks both against the O(N^2) direct sum.

usage: python scripts/bh_demo.py [--power 17] [--order 4] [--theta 0.6] [--ncrit 64] [--reps 5] [--direct 1]
"""

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from sphexa_amd.ops import gravity as G  # noqa: E402
from sphexa_amd.ops import octree as O  # noqa: E402
from sphexa_amd.ops import sfc  # noqa: E402
from sphexa_amd.utils.box import Box, OPEN  # noqa: E402


def cube_bodies(n, extent=3.0, seed=42):
    rng = np.random.default_rng(seed)
    X = rng.uniform(-extent, extent, (n, 3))
    X[0], X[-1] = -extent, extent
    m = rng.uniform(0, 1, n) / n
    h = np.full(n, np.cbrt(100.0 / n / 4.19) * extent)
    return X, m, h


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        r = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps, r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--power", type=int, default=17)
    ap.add_argument("--order", type=int, default=4)
    ap.add_argument("--theta", type=float, default=0.6)
    ap.add_argument("--ncrit", type=int, default=64)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--direct", type=int, default=1)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    n = (1 << a.power) - 1
    X, m_np, h_np = cube_bodies(n)
    box = Box([-3.0] * 3, [3.0] * 3, [OPEN] * 3)
    x, y, z = (torch.from_numpy(X[:, k].copy()).to(dev) for k in range(3))
    keys, perm = sfc.sort_keys(sfc.compute_keys(x, y, z, box))
    perm = perm.long()
    x, y, z = x[perm], y[perm], z[perm]
    m = torch.from_numpy(m_np).float().to(dev)[perm]
    h = torch.from_numpy(h_np).float().to(dev)[perm]

    t0 = time.perf_counter()
    tree, counts = O.update_tree(None, keys, a.ncrit)
    ot = O.build_octree(tree, counts, keys, x, y, z)
    centers, mp = G.upsweep(ot, x, y, z, m, box, a.theta)
    Q = G.multipole_upsweep(ot, centers, x, y, z, m, a.order)
    torch.cuda.synchronize()
    t_build = time.perf_counter() - t0

    acc = [torch.zeros(n, dtype=torch.float32, device=dev) for _ in range(3)]

    def run_p():
        for t in acc:
            t.zero_()
        return G.compute_gravity_multipole(ot, centers, Q, a.order, 0, n, x, y, z, h, m, 1.0, *acc)

    stats = {}

    def run_q():
        for t in acc:
            t.zero_()
        return G.compute_gravity(ot, centers, mp, 0, n, x, y, z, h, m, 1.0, *acc, stats=stats)

    t_p, e_p = timed(run_p, a.reps)
    ap_ = torch.stack(acc, 1).double().cpu()
    t_q, e_q = timed(run_q, a.reps)
    aq = torch.stack(acc, 1).double().cpu()
    out = {"bodies": n, "order": a.order, "theta": a.theta, "ncrit": a.ncrit, "leaves": int(counts.numel()),
           "build_upsweep_s": t_build, "bh_order_p_s": t_p, "bh_quadrupole_s": t_q,
           "p2p_per_body": stats.get("p2p", 0) / n, "m2p_per_body": stats.get("m2p", 0) / n}
    # reference demo.cu flop model: 20 per P2P, 2 P^3 per M2P (interaction counts of the production walk)
    flops = (out["p2p_per_body"] * 20 + out["m2p_per_body"] * 2 * a.order ** 3) * n
    out["tflops_order_p"] = flops / t_p / 1e12
    if a.direct:
        ref = [torch.zeros(n, dtype=torch.float32, device=dev) for _ in range(3)]
        e_d = G.direct_sum(0, n, x, y, z, h, m, 1.0, *ref)
        r = torch.stack(ref, 1).double().cpu()
        for name, v, e in (("order_p", ap_, e_p), ("quadrupole", aq, e_q)):
            rel = ((v - r).norm(dim=1) / r.norm(dim=1)).numpy()
            rel.sort()
            out[name + "_err"] = {"p50": float(rel[n // 2]), "p99": float(rel[int(0.99 * n)]),
                                  "max": float(rel[-1]), "energy": abs(e - e_d) / abs(e_d)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
