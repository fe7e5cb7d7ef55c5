"""All test cases and propagators step on the GPU (HIP path) and agree with the OpenMP path after one step;
turbulence stirring kernel vs CPU; Sedov CI accuracy (reference .jenkins/reframe_ci.py:255-353)."""

import math

import numpy as np
import pytest
import torch

from sphexa_amd.app.simulation import Simulation
from sphexa_amd.models.init import base as init_base
from sphexa_amd.models.init import cases

pytestmark = pytest.mark.gpu


@pytest.fixture
def small_glass(monkeypatch):
    blk = init_base.make_glass_block(8, relax_iters=10)
    monkeypatch.setattr(cases, "load_block", lambda path=None, n_side=16: blk)
    yield


def _sorted_state(sim, names):
    keys = sim.local("keys").cpu()
    order = torch.argsort(keys)
    return {n: sim.local(n).cpu()[order].double() for n in names}


@pytest.mark.parametrize("case,prop,n", [("noh", "ve", 32), ("evrard", "ve", 32), ("isobaric-cube", "ve", 32),
                                         ("gresho-chan", "ve", 8), ("noh", "std", 32), ("evrard", "nbody", 32),
                                         ("wind-shock", "ve", 8), ("kelvin-helmholtz", "ve", 8)])
def test_case_gpu_matches_cpu(gpu, small_glass, case, prop, n):
    cpu = Simulation(case, n=n, prop=prop, device="cpu")
    dev = Simulation(case, n=n, prop=prop, device=gpu)
    cpu.run(1)
    dev.run(1)
    assert abs(dev.d.minDt - cpu.d.minDt) <= 1e-4 * cpu.d.minDt
    names = ["x", "vx", "h"] + (["temp"] if prop != "nbody" else [])
    a, b = _sorted_state(cpu, names), _sorted_state(dev, names)
    # gravity: GPU (64-target groups) and CPU (16-target groups) traversals differ within the BH error
    tol = 2e-2 if case == "evrard" else 2e-4
    for k in names:
        scale = float(a[k].abs().max()) + 1e-30
        assert float((a[k] - b[k]).abs().max()) / scale < tol, k


def test_turbulence_gpu(gpu, small_glass):
    cpu = Simulation("turbulence", n=32, prop="turbulence", device="cpu")
    dev = Simulation("turbulence", n=32, prop="turbulence", device=gpu)
    cpu.run(2)
    dev.run(2)
    a, b = _sorted_state(cpu, ["vx", "vy"]), _sorted_state(dev, ["vx", "vy"])
    for k in a:
        assert float((a[k] - b[k]).abs().max()) / float(a[k].abs().max()) < 1e-3


@pytest.mark.slow
def test_sedov_ci_accuracy(gpu, tmp_path):
    """sedov grid -n 50 -s 200 (VE) L1 errors vs the self-similar solution.

    The reference CI (.jenkins/reframe_ci.py:350-353, a 2022 build) records density/pressure/velocity L1 of
    0.138/0.902/0.915 but not the simulation time reached after 200 steps, on which the errors depend strongly, so
    parity is unpinned: this is a regression guard on our own MI355X result (density 0.344, pressure 0.921,
    velocity 0.936 in the reference's comparison convention at t = 0.1155)."""
    from sphexa_amd.analysis.compare import l1_errors

    sim = Simulation("sedov", n=50, device=gpu)
    sim.run(200)
    d, s, e = sim.d, sim.domain.start_index(), sim.domain.end_index()
    from sphexa_amd.ops import hydro as H

    d.release("ax", "ay", "az")
    d.acquire("rho", "p", "gradh")
    H.compute_ve_def_gradh(d, sim.propagator.nl, sim.domain.box)
    H.compute_eos_ve(d, s, e)
    data = {k: d[k][s:e].double().cpu().numpy() for k in ("x", "y", "z", "vx", "vy", "vz", "rho", "p")}
    settings = sim.sim_init.constants()
    err = l1_errors(data, {"time": d.ttot}, settings, "sedov", reference_quirk=True)
    print("L1", err, "t", d.ttot)
    assert err["Density"] < 0.40
    assert abs(err["Pressure"] - 0.921) < 0.03 and abs(err["Velocity"] - 0.936) < 0.03
