#!/usr/bin/env python3
"""LET halo volume of the push-based multi-rank gravity at a given per-rank share, on CPU ranks over gloo (verdict
r4 item 8): python scripts/let_cost.py [-n 200] [--ranks 8]. Prints per rank the owned particles, SPH and gravity
halos (ratios to the owned count), remote multipoles and the M2P/P2P interactions per target."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-n", type=int, default=200)
    ap.add_argument("--ranks", type=int, default=8)
    a = ap.parse_args()
    from mp_util import run_ranks
    from test_multirank import _let_cost_worker

    t0 = time.time()
    res = run_ranks(_let_cost_worker, a.ranks, a.n)
    tot = sum(r["n"] for r in res)
    print(f"Evrard -n {a.n} on {a.ranks} CPU ranks ({tot} particles, {tot // a.ranks} per rank), "
          f"{time.time() - t0:.0f} s")
    print("| rank | owned | SPH halos | gravity halos | remote multipoles | local M2P / P2P per target | "
          "remote M2P / P2P per target |")
    print("|---|---|---|---|---|---|---|")
    for q, r in enumerate(res):
        print(f"| {q} | {r['n']} | {r['sph_halos']} ({r['sph_halos'] / r['n']:.2f}x) | {r['grav_halos']} "
              f"({r['grav_halos'] / r['n']:.2f}x) | {r['remote']} | {r['lm2p'] / r['n']:.0f} / {r['lp2p'] / r['n']:.0f} "
              f"| {r['rm2p'] / r['n']:.0f} / {r['rp2p'] / r['n']:.0f} |")
    g = [r["grav_halos"] / r["n"] for r in res]
    print(f"gravity halos / owned: mean {sum(g) / len(g):.2f}, max {max(g):.2f}")


if __name__ == "__main__":
    main()
