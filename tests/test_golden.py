"""Golden values of the SPH j-loops on the reference's own fixtures.

Reference: sph/test/ve.cpp:112-232 (99-particle fixture sph/test/example_data.txt, particle 0 against neighbors 1..98,
T = double) and sph/test/std.cpp:98-123 (5 particles). ``tests/data/sph_ve_fixture.txt`` is a verbatim copy of the
reference's data file (the GPU box has no /root/reference).

Three tiers:
  1. the j-loops of sph_math.hpp instantiated in double (_sphx_golden, built with -DSPHX_HYDRO_TYPE=double) against
     the reference's golden numbers at the reference's tolerances — this pins the formulas;
  2. the production fp32 OpenMP operators (ops/hydro.py) on the same inputs against tier 1 at fp32 tolerances;
  3. the production gfx950 operators (packed / fixed-point records) against tier 1 (``-m gpu``).
The fixture is in cgs units (m = 3.8e26 g, h = 1e7 cm): fp32 overflows in the IAD sums of that data (as the
reference's float build would), so tiers 2-3 run XMass/Gradh on the raw fixture and the remaining loops on a copy
with every field divided by a per-field scale (the j-loops are then evaluated on identical inputs by both tiers).
"""

import math
import os

import numpy as np
import pytest
import torch

from sphexa_amd.ops import _lib
from sphexa_amd.utils import kernel_tables

HERE = os.path.dirname(os.path.abspath(__file__))
COLS = ("x y z vx vy vz h c c11 c12 c13 c22 c23 c33 p gradh rho0 sumwhrho0 sumwh dvxdx dvxdy dvxdz dvydx dvydy dvydz "
        "dvzdx dvzdy dvzdz alpha u divv").split()
MPART = 3.781038064465603e26
SINC = 6.0


def sphynx_3d_k(n):
    """closed-form sinc^n normalization used by the reference tests (sph_kernel_tables.hpp:64-74)"""
    b0, b1, b2, b3 = 2.7012593e-2, 2.0410827e-2, 3.7451957e-3, 4.7013839e-2
    return b0 + b1 * math.sqrt(n) + b2 * n + b3 * math.sqrt(n ** 3)


K = sphynx_3d_k(SINC)


def _tables64():
    """20000-point kernel tables in double, sample positions in double (reference tabulateFunction with T=double)"""
    xs = np.arange(kernel_tables.TABLE_SIZE, dtype=np.float64) * (2.0 / (kernel_tables.TABLE_SIZE - 1))
    return (np.ascontiguousarray(kernel_tables.kernel_fn(0, SINC)(xs), dtype=np.float64),
            np.ascontiguousarray(kernel_tables.kernel_derivative_fn(0, SINC)(xs), dtype=np.float64))


@pytest.fixture(scope="module")
def fx():
    a = np.loadtxt(os.path.join(HERE, "data", "sph_ve_fixture.txt"))
    f = {c: np.ascontiguousarray(a[:, k]) for k, c in enumerate(COLS)}
    n = a.shape[0]
    f["m"] = np.full(n, MPART)
    f["xm"] = f["m"] / f["rho0"]
    f["kx"] = K * f["xm"] / f["h"] ** 3
    f["prho"] = f["p"] / (f["kx"] * f["m"] ** 2 * f["gradh"])
    # symmetrized velocity gradient (reference ve.cpp symmetrizeGradV)
    f["dV"] = [f["dvxdx"], f["dvxdy"] + f["dvydx"], f["dvxdz"] + f["dvzdx"], f["dvydy"], f["dvydz"] + f["dvzdy"],
               f["dvzdz"]]
    f["wh"], f["whd"] = _tables64()
    return f


BOX_VE = (-1.0e9, 1.0e9)


def g():
    return _lib.golden()


def _ci(f):
    return [f[c][0] for c in ("c11", "c12", "c13", "c22", "c23", "c33")]


# ------------------------------------------------------------------------- tier 1: fp64 j-loops vs golden numbers
def test_xmass_golden(fx):
    xm = g().xmass(K, *BOX_VE, fx["x"], fx["y"], fx["z"], fx["h"], fx["m"], fx["wh"], fx["whd"], SINC)
    rho0 = fx["m"][0] / xm
    assert rho0 == pytest.approx(34.515038498081417, abs=7.33e-7)
    assert abs(xm - fx["m"][0] / fx["rho0"][0]) <= fx["m"][0] / fx["rho0"][0] * 1e-7


def test_ve_def_gradh_golden(fx):
    kx, gradh = g().ve_def_gradh(K, *BOX_VE, fx["x"], fx["y"], fx["z"], fx["h"], fx["m"], fx["xm"], fx["wh"],
                                 fx["whd"], SINC)
    density = kx * fx["m"][0] / fx["xm"][0]
    assert density == pytest.approx(3.4662283566584293e1, abs=8e-7)
    assert gradh == pytest.approx(0.98699067585409861, abs=5e-7)
    assert kx == pytest.approx(1.0042661134076782, abs=3e-7)


def test_iad_golden(fx):
    c = g().iad(K, *BOX_VE, fx["x"], fx["y"], fx["z"], fx["h"], fx["xm"], fx["kx"], fx["wh"], fx["whd"], SINC)
    want = [1.9296619855715329e-18, -1.7838691836843698e-20, -1.2892885646884301e-20, 1.9482845913025683e-18,
            1.635410357476855e-20, 1.9246939006338132e-18]
    for got, w in zip(c, want):
        # the reference tolerance (1e-10 absolute) is vacuous for values ~1e-18; pin them to 1e-7 relative, the
        # level of the reference's other tolerances (XMass: 7.33e-7 on 34.5 = 2.1e-8 relative)
        assert got == pytest.approx(w, rel=1e-7)


def test_divv_curlv_golden(fx):
    divv, curlv, dV = g().divv_curlv(K, *BOX_VE, fx["x"], fx["y"], fx["z"], fx["vx"], fx["vy"], fx["vz"], fx["h"],
                                     _ci(fx), fx["kx"], fx["xm"], fx["wh"], fx["whd"], SINC)
    assert divv == pytest.approx(3.3760353440920682e-2, abs=2e-9)
    assert curlv == pytest.approx(3.7836647734377962e-2, abs=2e-9)
    want = [0.0013578323369918166, 0.02465266861727711, -0.0046604174274769167, 0.022556438947324862,
            0.0097704904179710741, 0.0098460821566040066]
    for got, w in zip(dV, want):
        assert got == pytest.approx(w, abs=2e-9)


def test_av_switches_golden(fx):
    alpha = g().av_switches(K, *BOX_VE, fx["x"], fx["y"], fx["z"], fx["vx"], fx["vy"], fx["vz"], fx["h"], fx["c"],
                            _ci(fx), fx["kx"], fx["xm"], fx["divv"], fx["wh"], fx["whd"], SINC, 0.3, 0.05, 1.0, 0.2,
                            fx["alpha"][0])
    assert alpha == pytest.approx(0.93941905320351171, abs=2e-9)


def _mom_args(f):
    return (f["x"], f["y"], f["z"], f["vx"], f["vy"], f["vz"], f["h"], f["c11"], f["c12"], f["c13"], f["c22"],
            f["c23"], f["c33"], f["m"], f["c"], f["xm"], f["kx"], f["prho"], f["alpha"], f["dV"], f["wh"], f["whd"],
            SINC)


@pytest.mark.parametrize("av_clean", [True, False])
def test_momentum_energy_golden(fx, av_clean):
    ax, ay, az, du, maxvs = g().momentum_energy(av_clean, K, 0.1, 0.2, *BOX_VE, *_mom_args(fx))
    if av_clean:
        want = [(-505548.68073726865, 0.023), (303384.91384746187, 0.053), (-1767463.9739728321, 0.043),
                (8.5525242525359648e12, 7.1e5)]
    else:
        want = [(-521261.07791667967, 0.022), (-74471.016515749841, 0.064), (-1730426.827721074, 0.042),
                (7.1838438980436924e12, 3.1e5)]
    for got, (w, tol) in zip((ax, ay, az, du), want):
        assert got == pytest.approx(w, abs=tol)
    assert maxvs == pytest.approx(26490876.319252387, abs=1e-6)


STD = dict(
    x=[1.0, 1.1, 3.2, 1.3, 2.4], y=[1.1, 1.2, 1.3, 4.4, 5.5], z=[1.2, 2.3, 1.4, 1.5, 1.6],
    h=[5.0, 5.1, 5.2, 5.3, 5.4], m=[1.1, 1.2, 1.3, 1.4, 1.5], rho=[0.014, 0.015, 0.016, 0.017, 0.018],
    vx=[0.010, -0.020, 0.030, -0.040, 0.050], vy=[-0.011, 0.021, -0.031, 0.041, -0.051],
    vz=[0.091, -0.081, 0.071, -0.061, 0.055], c=[0.4, 0.5, 0.6, 0.7, 0.8], p=[0.2, 0.3, 0.4, 0.5, 0.6],
    c11=[0.21, 0.27, 0.10, 0.45, 0.46], c12=[-0.22, -0.29, -0.11, -0.44, -0.47],
    c13=[-0.23, -0.31, -0.12, -0.43, -0.48], c22=[0.24, 0.32, 0.13, 0.42, 0.49],
    c23=[-0.25, -0.33, -0.14, -0.41, -0.50], c33=[0.26, 0.34, 0.15, 0.40, 0.51])
STD_IAD = [0.68826690779384281, -0.12963692768970825, -0.20435302538490346, 0.39616100688793993,
           -0.16797800827029263, 1.9055087813473524]
STD_MOM = [(14.407211846688075, 1.3e-7), (-1.2396802157028355, 1.4e-7), (15.596554152643426, 2.15e-7),
           (-0.40541191600274296, 1e-8)]
STD_VS = 1.4112466828564341


def _std():
    return {k: np.asarray(v, dtype=np.float64) for k, v in STD.items()}


def test_std_iad_golden(fx):
    s = _std()
    c = g().iad(K, 0.0, 6.0, s["x"], s["y"], s["z"], s["h"], s["m"], s["rho"], fx["wh"], fx["whd"], SINC)
    for got, w in zip(c, STD_IAD):
        assert got == pytest.approx(w, abs=1e-8)


def test_std_momentum_energy_golden(fx):
    s = _std()
    ax, ay, az, du, maxvs = g().momentum_energy_std(
        K, 0.0, 6.0, s["x"], s["y"], s["z"], s["vx"], s["vy"], s["vz"], s["h"], s["c11"], s["c12"], s["c13"],
        s["c22"], s["c23"], s["c33"], s["m"], s["rho"], s["p"], s["c"], fx["wh"], fx["whd"], SINC)
    for got, (w, tol) in zip((ax, ay, az, du), STD_MOM):
        assert got == pytest.approx(w, abs=tol)
    assert maxvs == pytest.approx(STD_VS, abs=1e-10)


# ---------------------------------------------------------------- tiers 2-3: production fp32 operators (CPU / GPU)
VE_FIELDS = ("x y z h m nc xm kx gradh vx vy vz c c11 c12 c13 c22 c23 c33 divv curlv alpha prho ax ay az du "
             "dV11 dV12 dV13 dV22 dV23 dV33").split()


def _dataset(dev, n, vals, fields=VE_FIELDS):
    from sphexa_amd.models import particles as P

    d = P.ParticlesData(dev)
    d.set_dependent(*fields)
    d.resize(n)
    d.K = K
    d.ng0, d.ngmax = min(50, n - 1), n - 1
    for k, v in vals.items():
        d[k] = torch.as_tensor(np.ascontiguousarray(v))
    d["nc"] = n  # particle 0 has every other particle as neighbor (count includes self)
    return d


def _neighbor_list(d, n):
    """particle 0 against 1..n-1 in the operator's list layout (CPU rows / GPU packed lists)"""
    from sphexa_amd.ops.neighbors import NeighborList, pack_lists

    k = np.arange(n - 1)
    if d.device.type == "cuda":
        return pack_lists([(k + 1).tolist()], 0, d.ngmax, d.device)
    return NeighborList(torch.from_numpy((k + 1).astype(np.int32)), 0, 1, d.ngmax, False)


def _box(lo, hi):
    from sphexa_amd.utils.box import Box, OPEN

    return Box([lo] * 3, [hi] * 3, [OPEN] * 3)


def _check_xmass_gradh(dev, f):
    from sphexa_amd.ops import hydro as H

    n = f["x"].size
    d = _dataset(dev, n, {c: f[c] for c in ("x", "y", "z", "h", "m")})
    nl = _neighbor_list(d, n)
    box = _box(*BOX_VE)
    H.compute_xmass(d, nl, box)
    rho0 = MPART / float(d["xm"][0])
    assert rho0 == pytest.approx(34.515038498081417, rel=2e-6)
    d["xm"] = f["xm"]
    H.compute_ve_def_gradh(d, nl, box)
    assert float(d["kx"][0]) == pytest.approx(1.0042661134076782, rel=2e-6)
    assert float(d["gradh"][0]) == pytest.approx(0.98699067585409861, rel=2e-6)


def _scaled(f):
    """every field divided by a per-field scale (fp32-safe magnitudes); the j-loops see identical inputs in all
    tiers. Coordinates and h share one scale so that r/h is unchanged."""
    L = f["h"][0]
    s = {c: f[c] / L for c in ("x", "y", "z", "h")}
    for grp in (("vx", "vy", "vz"), ("c",), ("c11", "c12", "c13", "c22", "c23", "c33"), ("m",), ("xm",), ("kx",),
                ("prho",), ("divv",)):
        scale = max(np.abs(np.concatenate([f[c] for c in grp])).max(), 1e-300)
        for c in grp:
            s[c] = f[c] / scale
    s["alpha"] = f["alpha"].copy()
    dvs = max(np.abs(np.concatenate(f["dV"])).max(), 1e-300)
    s["dV"] = [v / dvs for v in f["dV"]]
    s["wh"], s["whd"] = f["wh"], f["whd"]
    return s


def _check_scaled_loops(dev, f):
    from sphexa_amd.ops import hydro as H

    s = _scaled(f)
    n = s["x"].size
    box = (-1.0e9 / f["h"][0], 1.0e9 / f["h"][0])
    vals = {c: s[c] for c in ("x", "y", "z", "h", "m", "xm", "kx", "vx", "vy", "vz", "c", "c11", "c12", "c13", "c22",
                              "c23", "c33", "divv", "prho", "alpha")}
    for k, c in enumerate(("dV11", "dV12", "dV13", "dV22", "dV23", "dV33")):
        vals[c] = s["dV"][k]
    d = _dataset(dev, n, vals)
    nl = _neighbor_list(d, n)
    B = _box(*box)

    # fused IAD + divv/curlv against the fp64 IAD followed by the fp64 divv/curlv with that IAD
    c_ref = g().iad(K, *box, s["x"], s["y"], s["z"], s["h"], s["xm"], s["kx"], s["wh"], s["whd"], SINC)
    dv_ref = g().divv_curlv(K, *box, s["x"], s["y"], s["z"], s["vx"], s["vy"], s["vz"], s["h"], c_ref, s["kx"],
                            s["xm"], s["wh"], s["whd"], SINC)
    H.compute_iad_divv_curlv(d, nl, B, av_clean=True)
    cmax = max(abs(v) for v in c_ref)
    for k, c in enumerate(("c11", "c12", "c13", "c22", "c23", "c33")):
        assert abs(float(d[c][0]) - c_ref[k]) <= 2e-5 * cmax, c
    assert float(d["divv"][0]) == pytest.approx(dv_ref[0], rel=1e-5)
    assert float(d["curlv"][0]) == pytest.approx(dv_ref[1], rel=1e-5)
    dvmax = max(abs(v) for v in dv_ref[2])
    for k, c in enumerate(("dV11", "dV12", "dV13", "dV22", "dV23", "dV33")):
        assert abs(float(d[c][0]) - dv_ref[2][k]) <= 1e-5 * dvmax, c

    # AV switches and momentum/energy on the (scaled) fixture fields
    for k, c in enumerate(("c11", "c12", "c13", "c22", "c23", "c33")):
        d[c] = s[c]
    d["divv"] = s["divv"]
    for k, c in enumerate(("dV11", "dV12", "dV13", "dV22", "dV23", "dV33")):
        d[c] = s["dV"][k]
    d.minDt = 0.3
    a_ref = g().av_switches(K, *box, s["x"], s["y"], s["z"], s["vx"], s["vy"], s["vz"], s["h"], s["c"], _ci(s),
                            s["kx"], s["xm"], s["divv"], s["wh"], s["whd"], SINC, 0.3, 0.05, 1.0, 0.2, s["alpha"][0])
    H.compute_av_switches(d, nl, B)
    assert float(d["alpha"][0]) == pytest.approx(a_ref, rel=1e-5)
    d["alpha"] = s["alpha"]
    for av_clean in (True, False):
        ref = g().momentum_energy(av_clean, K, 0.1, 0.2, *box, *_mom_args(s))
        H.compute_momentum_energy_ve(d, nl, B, av_clean)
        amax = max(abs(v) for v in ref[:3])
        for k, c in enumerate(("ax", "ay", "az")):
            assert abs(float(d[c][0]) - ref[k]) <= 1e-5 * amax, (av_clean, c, float(d[c][0]), ref[k])
        assert float(d["du"][0]) == pytest.approx(ref[3], rel=1e-5)


def _check_std(dev, f):
    from sphexa_amd.ops import hydro as H

    s = _std()
    fields = "x y z h m nc rho p c vx vy vz c11 c12 c13 c22 c23 c33 ax ay az du".split()
    d = _dataset(dev, 5, {k: v for k, v in s.items()}, fields)
    nl = _neighbor_list(d, 5)
    B = _box(0.0, 6.0)
    c6 = [s[c].copy() for c in ("c11", "c12", "c13", "c22", "c23", "c33")]
    H.compute_iad(d, nl, B, "m", "rho")
    for k, c in enumerate(("c11", "c12", "c13", "c22", "c23", "c33")):
        assert float(d[c][0]) == pytest.approx(STD_IAD[k], rel=2e-6, abs=1e-7), c
    for k, c in enumerate(("c11", "c12", "c13", "c22", "c23", "c33")):
        d[c] = c6[k]
    H.compute_momentum_energy_std(d, nl, B)
    # acceleration components against the largest one (ay = -1.24 is a sum of terms of ~15 that nearly cancel: fp32
    # rounding of the analytic GPU kernel, ~1e-7 per term, is ~3e-6 of ay alone), du relative to itself
    amax = max(abs(w) for w, _ in STD_MOM[:3])
    for got, (w, _) in zip([float(d[c][0]) for c in ("ax", "ay", "az")], STD_MOM[:3]):
        assert abs(got - w) <= 5e-7 * amax
    assert float(d["du"][0]) == pytest.approx(STD_MOM[3][0], rel=2e-6, abs=1e-7)


def test_production_cpu_xmass_gradh(fx):
    _check_xmass_gradh("cpu", fx)


def test_production_cpu_scaled_loops(fx):
    _check_scaled_loops("cpu", fx)


def test_production_cpu_std(fx):
    _check_std("cpu", fx)


@pytest.mark.gpu
def test_production_gpu_xmass_gradh(fx, gpu):
    _check_xmass_gradh(gpu, fx)


@pytest.mark.gpu
def test_production_gpu_scaled_loops(fx, gpu):
    _check_scaled_loops(gpu, fx)


@pytest.mark.gpu
def test_production_gpu_std(fx, gpu):
    _check_std(gpu, fx)
