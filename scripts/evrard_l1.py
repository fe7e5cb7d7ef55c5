"""Evrard collapse on one GPU up to t/t* = 0.77 (and optionally 1.29): L1 errors of density, pressure and radial
velocity against the tabulated profiles (analysis/solutions.py: evrard_profiles; reference compare_evrard.py)."""
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from sphexa_amd.analysis.compare import l1_errors
from sphexa_amd.app.simulation import Simulation
from sphexa_amd.ops import hydro as H


def state(sim):
    d, s, e = sim.d, sim.domain.start_index(), sim.domain.end_index()
    d.release("ax", "ay", "az")
    d.acquire("rho", "p", "gradh")
    H.compute_ve_def_gradh(d, sim.propagator.nl, sim.domain.box)
    H.compute_eos_ve(d, s, e)
    data = {k: d[k][s:e].double().cpu().numpy() for k in ("x", "y", "z", "vx", "vy", "vz", "rho", "p")}
    d.release("rho", "p", "gradh")
    d.acquire("ax", "ay", "az")
    return data


n = int(sys.argv[1]) if len(sys.argv) > 1 else 50
targets = [float(v) for v in sys.argv[2:]] or [0.77]
sim = Simulation("evrard", n=n, device="cuda")
settings = sim.sim_init.constants()
res = {"n": n, "particles": int(sim.d.numParticlesGlobal), "results": []}
t0 = time.time()
steps = 0
for tt in targets:
    while sim.d.ttot + sim.d.minDt * 0.5 < tt:
        sim.step()
        steps += 1
        if steps % 200 == 0:
            print(f"step {steps} t {sim.d.ttot:.4f} dt {sim.d.minDt:.3g}", flush=True)
    err = l1_errors(state(sim), {"time": sim.d.ttot}, settings, "evrard")
    res["results"].append(dict(target=tt, t=sim.d.ttot, steps=steps, l1=err, wall_s=time.time() - t0))
    print(json.dumps(res["results"][-1]), flush=True)
json.dump(res, open(f"gpurun_out/evrard_l1_n{n}.json", "w"), indent=1)
