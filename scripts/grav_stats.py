#!/usr/bin/env python3
"""Gravity evaluation statistics of a case after a few steps: interactions per target, spilled groups and the share
of 64-source P2P chunks evaluated on the MFMA tile vs the VALU fallback (gravity.hip flushP2P), plus the pair-loop
frame code (ops/hydro.py fixed_point_code). usage: python scripts/grav_stats.py [--init evrard] [-n 200] [--steps 2]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from sphexa_amd.app.simulation import Simulation  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--init", default="evrard")
    ap.add_argument("-n", type=int, default=200)
    ap.add_argument("--steps", type=int, default=2)
    a = ap.parse_args()
    sim = Simulation(a.init, n=a.n)
    for _ in range(a.steps):
        sim.step()
    d = sim.d
    st = dict(sim.propagator.gravity.stats) if sim.propagator.gravity else {}
    n = sim.domain.end_index() - sim.domain.start_index()
    code = int(d.fixedPoint)
    shifts = [(code >> (1 + 5 * k)) & 31 for k in range(3)]
    print(f"case {a.init} -n {a.n}: {n} particles, frame code {code:#x} (shifts {shifts}), "
          f"h [{float(d['h'][:d.size].min()):.3e}, {float(d['h'][:d.size].max()):.3e}]")
    if st:
        mf, va = st.get("p2p_mfma_chunks", 0), st.get("p2p_valu_chunks", 0)
        print(f"P2P/target {st['p2p'] / n:.0f} (max {st['max_p2p']}), M2P/target {st['m2p'] / n:.0f} "
              f"(max {st['max_m2p']}), spilled groups {st['fallback']}, P2P chunks: MFMA {mf}, VALU {va} "
              f"({100.0 * va / max(mf + va, 1):.2f} % fallback)")


if __name__ == "__main__":
    main()
