#!/usr/bin/env python3
"""diagnostic: 1-rank vs 2-rank (one GPU, gloo) VE steps of Sedov -n 14, per-rank energies and the largest field
differences, with toggles of the round-4 changes (frame codes, global h extremes)"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import test_distributed_gpu as T  # noqa: E402


def main():
    n = 14
    for steps in (1, 2):
        ref = T._run(T._sph_worker, 1, n, steps)[0]
        res = T._run(T._sph_worker, 2, n, steps)
        keys = np.concatenate([r["keys"] for r in res])
        temp = np.concatenate([r["temp"] for r in res])
        o, ro = np.argsort(keys), np.argsort(ref["keys"])
        dT = np.abs(temp[o] - ref["temp"][ro]).max() / np.abs(ref["temp"]).max()
        print(f"steps {steps}: etot 1 rank {ref['etot']:.10g}, 2 ranks {res[0]['etot']:.10g} / {res[1]['etot']:.10g}; "
              f"dt {ref['dt']:.6g} vs {res[0]['dt']:.6g}; nsum {ref['nsum']} vs {res[0]['nsum']}; max temp diff {dT:.3e}")


if __name__ == "__main__":
    main()
