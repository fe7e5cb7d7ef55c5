"""Noh implosion -n 50 (VE, built-in glass) L1 errors vs the analytical solution at several steps (the reference CI
runs -n 50 -s 200 with its glass.h5 and checks density/pressure/velocity L1 = 10.42/2.88/0.14, .gitlab/rfm.py:48-53).
usage: python scripts/noh_l1.py [n] [steps...]"""
import json
import sys

import torch

sys.path.insert(0, ".")
from sphexa_amd.analysis.compare import l1_errors  # noqa: E402
from sphexa_amd.app.simulation import Simulation  # noqa: E402
from sphexa_amd.ops import hydro as H  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    marks = [int(v) for v in sys.argv[2:]] or [100, 200]
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    sim = Simulation("noh", n=n, device=dev, quiet=True)
    settings = sim.sim_init.constants()
    out, done = [], 0
    for m in marks:
        sim.run(m - done)
        done = m
        d, s, e = sim.d, sim.domain.start_index(), sim.domain.end_index()
        d.release("ax", "ay", "az")
        d.acquire("rho", "p", "gradh")
        H.compute_ve_def_gradh(d, sim.propagator.nl, sim.domain.box)
        H.compute_eos_ve(d, s, e)
        data = {k: d[k][s:e].double().cpu().numpy() for k in ("x", "y", "z", "vx", "vy", "vz", "rho", "p")}
        d.release("rho", "p", "gradh")
        d.acquire("ax", "ay", "az")
        err = l1_errors(data, {"time": d.ttot}, settings, "noh")
        out.append({"step": m, "time": d.ttot, **err})
        print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    main()
