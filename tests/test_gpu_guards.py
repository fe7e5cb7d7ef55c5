"""GPU tier: failure detection and the precision guard of the pair-loop records.

* The coupled nc/h iteration raises when it does not converge (reference sph/hydro_ve/xmass_gpu.cu:82-92,131).
* Evrard (open, collapsing cloud, hmin/hmed ~ 0.1) runs the pair loops on fp64-coordinate records under the
  2^-22 guard (ops/hydro.py: fixed_point_ok); forcing the fixed-point records on the same state shows how far they
  are from the fp64 path on a high-dynamic-range case.
"""

import pytest
import torch

from sphexa_amd.ops import hydro as H

pytestmark = pytest.mark.gpu


def test_gpu_h_iteration_failure_raises(gpu, monkeypatch):
    from sphexa_amd.models import particles as P
    from sphexa_amd.ops import neighbors as N
    from sphexa_amd.ops import octree as O
    from sphexa_amd.ops import sfc
    from sphexa_amd.utils.box import Box, PERIODIC

    box = Box.cube(0.0, 1.0, PERIODIC)
    g = torch.Generator().manual_seed(4)
    X = torch.rand(30, 3, generator=g, dtype=torch.float64).to(gpu)
    d = P.ParticlesData(gpu)
    d.set_conserved("x", "y", "z", "h", "m")
    d.set_dependent("nc", "keys")
    d.resize(30)
    keys = sfc.compute_keys(X[:, 0].contiguous(), X[:, 1].contiguous(), X[:, 2].contiguous(), box)
    s, p = sfc.sort_keys(keys)
    for k, c in enumerate("xyz"):
        d[c] = X[p, k].contiguous()
    d["h"] = 0.05
    d.ng0, d.ngmax = 200, 250
    tree, counts = O.update_tree(None, s, 16)
    ot = O.build_octree(tree, counts, s, d["x"], d["y"], d["z"])
    with pytest.raises(N.NeighborSearchError, match="failed to converge"):
        N.find_neighbors(d, ot, box, 0, d.size, iterate_h=True)
    monkeypatch.setattr(N, "ALLOW_NC_FAIL", True)
    d["h"] = 0.05
    N.find_neighbors(d, ot, box, 0, d.size, iterate_h=True)
    assert d.nc_fail > 0


def _evrard_step(gpu, force):
    """one Evrard step; ``force``: None (natural frame), or the frame code every pair loop takes (0: fp64 records,
    1: unshifted 32-bit box frame)"""
    from sphexa_amd.app.simulation import Simulation

    sim = Simulation("evrard", n=40, device=gpu)
    h = sim.d["h"][: sim.d.size]
    natural = H.frame_code(sim.domain.box, float(h.min()), float(h.max()))
    if force is not None:
        orig = H.fixed_point_code
        H.fixed_point_code = lambda d, box: force
    try:
        sim.step()
        code = sim.d.fixedPoint
    finally:
        if force is not None:
            H.fixed_point_code = orig
    s, e = sim.domain.start_index(), sim.domain.end_index()
    return natural, code, {f: sim.d[f][s:e].double().cpu() for f in ("ax", "ay", "az", "du", "alpha", "h")}


def test_evrard_frame_shift_keeps_fixed_point_records(gpu):
    """Evrard's collapsing cloud: the unshifted box frame (quanta of L/2^31) is too coarse for its smallest h, the
    shifted frame (wrap period L/2^k > 4.5 h_max, sph_math.hpp qframeOf) is not: the pair loops keep the 32-bit
    records, and their forces match the fp64-coordinate records"""
    natural, code, ref = _evrard_step(gpu, None)
    shifts = [(natural >> (1 + 5 * k)) & 31 for k in range(3)]
    print(f"Evrard n=40: frame code {natural:#x}, shifts {shifts}")
    assert natural != 0 and code == natural and min(shifts) > 0
    _, c64, f64 = _evrard_step(gpu, 0)
    assert c64 == 0
    for f, tol in (("ax", 2e-6), ("ay", 2e-6), ("az", 2e-6), ("du", 2e-6), ("alpha", 1e-6)):
        scale = max(f64[f].abs().max().item(), 1e-30)  # du is 0 on the first step of the cloud at rest
        err = (ref[f] - f64[f]).abs().max().item() / scale
        print(f"shifted fixed-point vs fp64 records, {f}: max |diff| / max |fp64| = {err:.3e}")
        assert err < tol, (f, err)


def test_evrard_unshifted_frame_stays_close(gpu):
    """the unshifted box frame, forced below its quantum bound, is still within fp32-level distance of fp64"""
    _, c1, fx = _evrard_step(gpu, 1)
    _, _, f64 = _evrard_step(gpu, 0)
    assert c1 == 1
    for f, tol in (("ax", 2e-4), ("ay", 2e-4), ("du", 2e-4), ("alpha", 1e-5)):
        scale = max(f64[f].abs().max().item(), 1e-30)
        err = (fx[f] - f64[f]).abs().max().item() / scale
        print(f"unshifted fixed-point vs fp64 records, {f}: max rel err {err:.3e}")
        assert err < tol, (f, err)


@pytest.mark.parametrize("mode", ["clean", "corrupt"])
def test_device_check_build(mode):
    """device-check HIP build (build_native --dcheck, SPHX_DEVICE_CHECKS=1): range checks in the pair loops, gathers,
    halo packing and gravity lists report a corrupted input after the step instead of faulting (common.h)"""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, SPHX_DEVICE_CHECKS="1")
    env.pop("SPHX_HIP_VARIANT", None)
    p = subprocess.run([sys.executable, os.path.join(root, "tests", "helpers", "dcheck_run.py"), mode], env=env,
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    if mode == "clean":
        assert "clean ok" in p.stdout
    else:
        assert "caught: device checks failed in corrupted list: neighbor index out of range" in p.stdout
