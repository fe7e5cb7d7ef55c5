#!/usr/bin/env python3
"""Micro-benchmarks that mirror the reference's performance drivers (fixed roofline anchors for the search, octree and
SFC-sort kernels), timed with device events after one untimed call:

  hilbert   domain/test/performance/hilbert.cu:77-180     32 M uniform keys in [-1,1]^3: Hilbert key computation,
                                                           sort of the random keys, and the re-sort of slightly moved
                                                           keys (the per-step case of an SPH run)
  octree    domain/test/performance/octree.cu:72-116      2 M Gaussian particles (sigma = box/5, clamped), bucket 16:
                                                           cornerstone leaf build from scratch, update with the previous
                                                           tree as guess, fully linked octree (internal nodes, ranges,
                                                           boxes)
  neighbors domain/test/performance/neighbor_driver.cu:174-280  2 M uniform periodic particles, h = 0.012, ngmax = 200,
                                                           bucket 64: GPU search (fixed h) -> pairs/s

usage: python scripts/micro_bench.py [hilbert|octree|neighbors ...] [--reps R]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from sphexa_amd.ops import octree as O  # noqa: E402
from sphexa_amd.ops import sfc  # noqa: E402
from sphexa_amd.utils.box import Box, OPEN, PERIODIC  # noqa: E402

DEV = torch.device("cuda", 0)


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return min(ts), float(np.median(ts))


def bench_hilbert(reps):
    n = 32_000_000
    g = torch.Generator(device=DEV).manual_seed(0)
    x, y, z = (torch.rand(n, generator=g, device=DEV, dtype=torch.float64) * 2 - 1 for _ in range(3))
    box = Box.cube(-1.0, 1.0, OPEN)
    keys = torch.empty(n, dtype=torch.int64, device=DEV)
    t_keys = timed(lambda: sfc.compute_keys(x, y, z, box, sfc.HILBERT, out=keys), reps)
    t_rand = timed(lambda: sfc.sort_keys(keys), reps)
    s, p = sfc.sort_keys(keys)
    # the per-step case: the sorted particles move by a small fraction of their spacing, keys recomputed in that order
    xs, ys, zs = x[p.long()], y[p.long()], z[p.long()]
    eps = 0.1 * 2.0 / n ** (1 / 3)
    moved = [c + eps * (torch.rand(n, generator=g, device=DEV, dtype=torch.float64) - 0.5) for c in (xs, ys, zs)]
    k2 = sfc.compute_keys(*[c.clamp(-1, 1) for c in moved], box, sfc.HILBERT)
    t_near = timed(lambda: sfc.sort_keys(k2), reps)
    s2, p2 = sfc.sort_keys(k2)
    assert bool((s2[1:] >= s2[:-1]).all())
    return {"driver": "hilbert.cu", "n": n, "hilbert_keys_ms": t_keys[0], "keys_per_s": n / t_keys[0] * 1e3,
            "sort_random_ms": t_rand[0], "sort_random_keys_per_s": n / t_rand[0] * 1e3,
            "sort_nearly_sorted_ms": t_near[0], "sort_nearly_sorted_keys_per_s": n / t_near[0] * 1e3,
            "median_ms": {"keys": t_keys[1], "sort_random": t_rand[1], "sort_nearly_sorted": t_near[1]}}


def bench_octree(reps):
    n, bucket = 2_000_000, 16
    rng = np.random.default_rng(0)
    X = np.clip(rng.normal(0.0, 2.0 / 5, (n, 3)), -1, 1)
    box = Box.cube(-1.0, 1.0, OPEN)
    x, y, z = (torch.from_numpy(X[:, k].copy()).to(DEV) for k in range(3))
    keys, p = sfc.sort_keys(sfc.compute_keys(x, y, z, box, sfc.MORTON))
    x, y, z = x[p.long()], y[p.long()], z[p.long()]
    t_scratch = timed(lambda: O.update_tree(None, keys, bucket, max_iter=64), reps)
    tree, counts = O.update_tree(None, keys, bucket, max_iter=64)
    t_update = timed(lambda: O.update_tree(tree, keys, bucket), reps)
    t_link = timed(lambda: O.build_octree(tree, counts, keys, x, y, z), reps)
    ot = O.build_octree(tree, counts, keys, x, y, z)
    return {"driver": "octree.cu", "n": n, "bucket": bucket, "leaves": ot.num_leaves, "nodes": ot.num_nodes,
            "build_from_scratch_ms": t_scratch[0], "update_with_guess_ms": t_update[0],
            "fully_linked_octree_ms": t_link[0],
            "median_ms": {"scratch": t_scratch[1], "update": t_update[1], "link": t_link[1]}}


def bench_neighbors(reps):
    from sphexa_amd.models import particles as P
    from sphexa_amd.ops.neighbors import find_neighbors

    n, h, ngmax = 2_000_000, 0.012, 200
    box = Box.cube(0.0, 1.0, PERIODIC)
    g = torch.Generator(device=DEV).manual_seed(1)
    d = P.ParticlesData(DEV)
    d.set_conserved("x", "y", "z", "h", "m")
    d.set_dependent("nc", "keys")
    d.resize(n)
    xyz = [torch.rand(n, generator=g, device=DEV, dtype=torch.float64) for _ in range(3)]
    keys, p = sfc.sort_keys(sfc.compute_keys(*xyz, box, sfc.HILBERT))
    for c, v in zip("xyz", xyz):
        d[c] = v[p.long()]
    d["h"] = h
    d["m"] = 1.0 / n
    d["keys"] = keys
    d.ng0, d.ngmax = 100, ngmax
    tree, counts = O.update_tree(None, keys, 64, max_iter=64)
    ot = O.build_octree(tree, counts, keys, d["x"], d["y"], d["z"])
    state = {}

    def run():
        state["nl"] = find_neighbors(d, ot, box, 0, n, iterate_h=False, prev=state.get("nl"))

    t = timed(run, reps)
    pairs = float((d["nc"].to(torch.float64) - 1).sum())
    return {"driver": "neighbor_driver.cu", "n": n, "h": h, "ngmax": ngmax, "mean_neighbors": pairs / n,
            "search_ms": t[0], "pairs_per_s": pairs / t[0] * 1e3, "median_ms": t[1]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("which", nargs="*", default=["hilbert", "octree", "neighbors"])
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    fns = {"hilbert": bench_hilbert, "octree": bench_octree, "neighbors": bench_neighbors}
    for w in args.which:
        print(json.dumps(fns[w](args.reps)), flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
