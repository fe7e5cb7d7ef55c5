"""Diagnose the Sedov -n 50 density L1 (VE, 200 steps): dt history, shock position vs the similarity solution,
radial density profile, L1 vs time."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from sphexa_amd.analysis import solutions as S
from sphexa_amd.analysis.compare import l1_errors
from sphexa_amd.app.simulation import Simulation
from sphexa_amd.ops import hydro as H


def snapshot(sim):
    d, s, e = sim.d, sim.domain.start_index(), sim.domain.end_index()
    d.release("ax", "ay", "az")
    d.acquire("rho", "p", "gradh")
    H.compute_ve_def_gradh(d, sim.propagator.nl, sim.domain.box)
    H.compute_eos_ve(d, s, e)
    data = {k: d[k][s:e].double().cpu().numpy() for k in ("x", "y", "z", "vx", "vy", "vz", "rho", "p", "h")}
    d.release("rho", "p", "gradh")
    d.acquire("ax", "ay", "az")
    return data


prop = sys.argv[1] if len(sys.argv) > 1 else "ve"
sim = Simulation("sedov", n=50, prop=prop, device="cuda")
settings = sim.sim_init.constants()
sol = S.SedovSolution(3, settings["gamma"])
hist = []
out = {"prop": prop, "l1": []}
for step in range(1, 201):
    sim.step()
    hist.append((step, sim.d.ttot, sim.d.minDt))
    if step % 25 == 0 and prop == "ve":
        data = snapshot(sim)
        err = l1_errors(data, {"time": sim.d.ttot}, settings, "sedov", reference_quirk=True)
        r = np.sqrt(data["x"] ** 2 + data["y"] ** 2 + data["z"] ** 2)
        bins = np.linspace(0, 0.6, 61)
        idx = np.digitize(r, bins)
        prof = [float(data["rho"][idx == k].mean()) if (idx == k).any() else 0.0 for k in range(1, 61)]
        rs = sol.shock_radius(sim.d.ttot)
        rpk = float(0.5 * (bins[np.argmax(prof)] + bins[np.argmax(prof) + 1]))
        out["l1"].append(dict(step=step, t=sim.d.ttot, dt=sim.d.minDt, l1=err, shock_exact=rs, rho_peak_r=rpk,
                              rho_peak=max(prof), hmean=float(data["h"].mean())))
        print(json.dumps(out["l1"][-1]), flush=True)
out["dt_history"] = hist[:20] + hist[20::10]
json.dump(out, open(f"gpurun_out/sedov_diag_{prop}.json", "w"), indent=1)
