#!/usr/bin/env python3
"""Inventory of the host synchronizations of one time step (torch sync-debug mode): which lines of the package copy
device values to the host, per step. usage: python scripts/sync_inventory.py [--init evrard] [-n 50]"""
import argparse
import collections
import os
import sys
import traceback
import warnings

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--init", default="evrard")
    ap.add_argument("-n", type=int, default=50)
    args = ap.parse_args()
    from sphexa_amd.app.simulation import Simulation

    sim = Simulation(args.init, n=args.n, prop="ve", device=torch.device("cuda", 0), out=None, quiet=True)
    sim.run(2)
    sites = collections.Counter()

    def hook(message, category, filename, lineno, file=None, line=None):
        for fr in reversed(traceback.extract_stack()[:-1]):
            if "sphexa_amd" in fr.filename:
                sites[f"{os.path.relpath(fr.filename)}:{fr.lineno} {fr.line}"] += 1
                break

    warnings.showwarning = hook
    warnings.simplefilter("always")
    torch.cuda.set_sync_debug_mode("warn")
    sim.run(1)
    torch.cuda.set_sync_debug_mode("default")
    print(f"{sum(sites.values())} synchronizing calls in one step ({args.init} -n {args.n}):")
    for k, v in sites.most_common():
        print(f"{v:4d}  {k}")


if __name__ == "__main__":
    main()
