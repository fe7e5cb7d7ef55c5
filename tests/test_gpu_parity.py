"""HIP kernels vs the OpenMP reference path (same inputs, same algorithms) — the GPU tier of the oracle tests.

Parity model: reference domain/test/unit_cuda/* (GPU vs CPU equality for keys, csarray, octree) and
sph/test (kernel j-loops). Tolerances: exact for integer data (keys, trees, neighbor sets), ~1e-5 relative for fp32
fields whose sums differ only in summation order.
"""

import math

import numpy as np
import pytest
import torch

from sphexa_amd.models import particles as P
from sphexa_amd.models.init.sedov import SedovGrid
from sphexa_amd.models.propagators import HydroVeProp, HydroProp
from sphexa_amd.ops import hydro as H
from sphexa_amd.ops import octree as O
from sphexa_amd.ops import sfc
from sphexa_amd.ops.neighbors import find_neighbors, neighbor_lists_as_sets
from sphexa_amd.parallel.comm import Comm
from sphexa_amd.parallel.domain import Domain
from sphexa_amd.utils.box import Box, OPEN, PERIODIC

pytestmark = pytest.mark.gpu


def _setup(device, n=16, prop_cls=HydroVeProp, jitter=0.0):
    d = P.ParticlesData(device)
    prop = prop_cls(None, 0)
    prop.activate_fields(d)
    box = SedovGrid().init(0, 1, n, d)
    if jitter:
        g = torch.Generator().manual_seed(7)
        for c in ("x", "y", "z"):
            d[c] = d[c].cpu() + jitter * (torch.rand(d.size, generator=g, dtype=torch.float64) - 0.5)
    dom = Domain(Comm(), box)
    return d, prop, dom


def _rel(a, b):
    a = a.detach().cpu().double()
    b = b.detach().cpu().double()
    scale = max(b.abs().max().item(), 1e-30)
    return (a - b).abs().max().item() / scale


def _check(g, c, fields, tol):
    """max |GPU - OpenMP| / max |OpenMP| per field (printed), each below ``tol``"""
    errs = {f: _rel(g[f], c[f]) for f in fields}
    print("GPU vs OpenMP:", {f: f"{e:.2e}" for f, e in errs.items()})
    for f, e in errs.items():
        assert e < tol, (f, e)


def test_device_is_gfx950(gpu):
    from sphexa_amd.ops import _lib

    info = _lib.hip().device_info()
    assert "gfx950" in info["arch"], info


def test_keys_and_sort(gpu):
    n = 100000
    g = torch.Generator().manual_seed(1)
    x, y, z = (torch.rand(n, generator=g, dtype=torch.float64) for _ in range(3))
    box = Box.cube(0.0, 1.0, OPEN)
    for kind in (sfc.HILBERT, sfc.MORTON):
        kc = sfc.compute_keys(x, y, z, box, kind)
        kg = sfc.compute_keys(x.to(gpu), y.to(gpu), z.to(gpu), box, kind)
        assert torch.equal(kc, kg.cpu())
        sc, pc = sfc.sort_keys(kc)
        sg, pg = sfc.sort_keys(kg)
        assert torch.equal(sc, sg.cpu())
        assert torch.equal(pc, pg.cpu().to(pc.dtype))


def test_gather_multi(gpu):
    n = 5000
    perm = torch.randperm(n, dtype=torch.int64).to(torch.int32)
    a = torch.rand(n, dtype=torch.float64)
    b = torch.rand(n, dtype=torch.float32)
    c = torch.arange(n, dtype=torch.int32)
    outs = sfc.gather_many(perm.to(gpu), [a.to(gpu), b.to(gpu), c.to(gpu)])
    for src, o in zip((a, b, c), outs):
        assert torch.equal(src[perm.long()], o.cpu())


def test_octree_build_and_link(gpu):
    n = 200000
    g = torch.Generator().manual_seed(3)
    x, y, z = (torch.randn(n, generator=g, dtype=torch.float64) * 0.1 + 0.5 for _ in range(3))
    box = Box.cube(-0.5, 1.5, OPEN)
    keys = sfc.sort_keys(sfc.compute_keys(x, y, z, box))[0]
    tc, cc = O.update_tree(None, keys, 64)
    tg, cg = O.update_tree(None, keys.to(gpu), 64)
    assert torch.equal(tc, tg.cpu())
    assert torch.equal(cc, cg.cpu())
    assert int(cc.max()) <= 64
    perm = sfc.sort_keys(sfc.compute_keys(x, y, z, box))[1].long()
    xs, ys, zs = x[perm], y[perm], z[perm]
    oc = O.build_octree(tc, cc, keys, xs, ys, zs)
    og = O.build_octree(tg, cg, keys.to(gpu), xs.to(gpu), ys.to(gpu), zs.to(gpu))
    assert oc.num_nodes == og.num_nodes
    for f in ("prefixes", "child_offsets", "node_to_leaf", "leaf_to_node", "node_start", "node_end", "parents"):
        assert torch.equal(getattr(oc, f), getattr(og, f).cpu()), f
    assert oc.level_range == og.level_range
    assert torch.allclose(oc.center, og.center.cpu())
    assert torch.allclose(oc.half, og.half.cpu())


@pytest.mark.parametrize("periodic", [True, False])
def test_neighbors_match_cpu(gpu, periodic):
    dc, pc, domc = _setup("cpu", 16, jitter=0.01)
    dg, pg, domg = _setup(gpu, 16, jitter=0.01)
    if not periodic:
        for dm in (domc, domg):
            dm.box.bc = [OPEN] * 3
    pc.sync(domc, dc)
    pg.sync(domg, dg)
    assert torch.equal(dc["keys"], dg["keys"].cpu())
    nlc = find_neighbors(dc, domc.octree, domc.box, 0, dc.size)
    nlg = find_neighbors(dg, domg.octree, domg.box, 0, dg.size)
    assert torch.equal(dc["nc"], dg["nc"].cpu())
    assert torch.allclose(dc["h"], dg["h"].cpu())
    sc = neighbor_lists_as_sets(nlc, dc["nc"])
    sg = neighbor_lists_as_sets(nlg, dg["nc"])
    assert sc == sg


@pytest.mark.parametrize("av_clean", [False, True])
def test_ve_step_matches_cpu(gpu, av_clean):
    results = {}
    for dev in ("cpu", gpu):
        d = P.ParticlesData(dev)
        prop = HydroVeProp(None, 0, av_clean=av_clean)
        prop.activate_fields(d)
        box = SedovGrid().init(0, 1, 16, d)
        dom = Domain(Comm(), box)
        prop.sync(dom, d)
        for _ in range(2):
            prop.step(dom, d)
            d.iteration += 1
        results[str(dev)] = {f: d[f].clone().cpu() for f in
                             ("x", "y", "z", "vx", "vy", "vz", "temp", "h", "alpha", "du", "ax", "c11", "xm", "kx",
                              "nc")}
        results[str(dev)]["dt"] = d.minDt
    c, g = results["cpu"], results[str(gpu)]
    assert math.isclose(c["dt"], g["dt"], rel_tol=1e-5)
    assert torch.equal(c["nc"], g["nc"])
    for f in ("x", "y", "z", "temp", "h", "xm", "kx", "c11", "alpha"):
        assert _rel(g[f], c[f]) < 2e-5, f
    _check(g, c, ("vx", "vy", "vz", "ax", "du"), 2e-5)


def test_std_step_matches_cpu(gpu):
    results = {}
    for dev in ("cpu", gpu):
        d = P.ParticlesData(dev)
        prop = HydroProp(None, 0)
        prop.activate_fields(d)
        box = SedovGrid().init(0, 1, 16, d)
        dom = Domain(Comm(), box)
        prop.sync(dom, d)
        prop.step(dom, d)
        results[str(dev)] = {f: d[f].clone().cpu() for f in ("x", "temp", "rho", "p", "ax", "du")}
    c, g = results["cpu"], results[str(gpu)]
    for f in ("x", "temp", "rho", "p"):
        assert _rel(g[f], c[f]) < 2e-5, f
    _check(g, c, ("ax", "du"), 2e-5)


def test_conserved_quantities(gpu):
    from sphexa_amd.models.observables import local_conserved

    q = {}
    for dev in ("cpu", gpu):
        d = P.ParticlesData(dev)
        prop = HydroVeProp(None, 0)
        prop.activate_fields(d)
        SedovGrid().init(0, 1, 12, d)
        d["vx"] = torch.linspace(-1, 1, d.size)
        d["nc"] = 7
        q[str(dev)] = local_conserved(d, 0, d.size).cpu()
    assert torch.allclose(q["cpu"], q[str(gpu)], rtol=1e-10, atol=1e-14)


def test_neighbor_spill_path(gpu, monkeypatch):
    """groups whose LDS frontier overflows are redone by the global-memory spill kernel with identical results"""
    from sphexa_amd.ops import neighbors as N

    dg, pg, domg = _setup(gpu, 16, jitter=0.01)
    pg.sync(domg, dg)
    h0 = dg["h"].clone()
    nl_ref = find_neighbors(dg, domg.octree, domg.box, 0, dg.size)
    nc_ref, h_ref = dg["nc"].clone(), dg["h"].clone()
    sets_ref = neighbor_lists_as_sets(nl_ref, nc_ref)
    dg["h"].copy_(h0)
    monkeypatch.setattr(N, "TEST_FRONT_CAP", 16)
    nl = find_neighbors(dg, domg.octree, domg.box, 0, dg.size)
    assert dg.nc_spilled > 0
    assert torch.equal(dg["nc"], nc_ref) and torch.equal(dg["h"], h_ref)
    assert neighbor_lists_as_sets(nl, dg["nc"]) == sets_ref


def test_neighbor_chunk_overflow_halves_h(gpu):
    """an initial h seven times too large makes the groups' candidates span more chunks than their tables hold (64 000
    lattice particles, ~34 000 per sphere): the search halves h for those groups and iterates on instead of failing,
    and the final lists are exactly the neighbor sets of the final h (CPU search, no iteration)"""
    from sphexa_amd.ops import neighbors as N

    dg, pg, domg = _setup(gpu, 40, jitter=0.01)
    pg.sync(domg, dg)
    n = dg.size
    dg["h"].mul_(7.0)
    with pytest.raises(N.NeighborSearchError, match="chunk"):
        find_neighbors(dg, domg.octree, domg.box, 0, n, iterate_h=False)
    nl = find_neighbors(dg, domg.octree, domg.box, 0, n)
    assert dg.nc_shrunk > (n + 63) // 128
    nc = dg["nc"].cpu()
    assert int(nc.min()) >= dg.ng0 // 4 and int(nc.max()) <= dg.ngmax + 1
    # CPU reference: the same particles, the GPU's final h, no h iteration
    dc, pc, domc = _setup("cpu", 40, jitter=0.01)
    pc.sync(domc, dc)
    assert torch.equal(dc["keys"], dg["keys"].cpu())
    dc["h"] = dg["h"].cpu()
    nl_c = find_neighbors(dc, domc.octree, domc.box, 0, n, iterate_h=False)
    assert torch.equal(dc["nc"], nc)
    assert neighbor_lists_as_sets(nl, dg["nc"]) == neighbor_lists_as_sets(nl_c, dc["nc"])


@pytest.mark.parametrize("case", ["lattice", "glass_evrard"])
def test_neighbor_subgroup_passes(gpu, monkeypatch, case):
    """target-group splitting: groups searched as sub-group passes of 16 lanes (each with its own search box, one
    shared chunk table) give the same h iteration, counts and neighbor sets as whole-group passes"""
    from sphexa_amd.app.simulation import Simulation
    from sphexa_amd.ops import neighbors as N

    if case == "lattice":
        dg, pg, domg = _setup(gpu, 16, jitter=0.01)
        pg.sync(domg, dg)
        tree, box, n = domg.octree, domg.box, dg.size
    else:
        sim = Simulation("evrard", n=30, device=gpu)
        dg, tree, box, n = sim.d, sim.domain.octree, sim.domain.box, sim.d.size
    h0 = dg["h"].clone()
    nl_ref = find_neighbors(dg, tree, box, 0, n)
    nc_ref, h_ref = dg["nc"].clone(), dg["h"].clone()
    sets_ref = neighbor_lists_as_sets(nl_ref, nc_ref)
    assert dg.nc_split == 0 or case != "lattice"
    dg["h"].copy_(h0)
    monkeypatch.setattr(N, "TEST_FORCE_SPLIT", True)
    nl = find_neighbors(dg, tree, box, 0, n)
    assert dg.nc_split == (n + 63) // 64
    assert torch.equal(dg["nc"], nc_ref) and torch.equal(dg["h"], h_ref)
    assert neighbor_lists_as_sets(nl, dg["nc"]) == sets_ref


@pytest.mark.parametrize("case", ["lattice", "glass_evrard"])
def test_neighbor_split_prediction(gpu, monkeypatch, case):
    """overflow prediction (neighbors.hip PredOut): the groups the main kernel had to queue are recorded by SFC key
    range; the next search hands them to the split kernel on a second stream, its main kernel queues fewer groups, and
    h, counts and neighbor sets stay those of the search without prediction"""
    from sphexa_amd.app.simulation import Simulation
    from sphexa_amd.ops import neighbors as N

    if case == "lattice":
        dg, pg, domg = _setup(gpu, 16, jitter=0.01)
        pg.sync(domg, dg)
        tree, box, n = domg.octree, domg.box, dg.size
    else:
        sim = Simulation("evrard", n=30, device=gpu)
        dg, tree, box, n = sim.d, sim.domain.octree, sim.domain.box, sim.d.size
    monkeypatch.setattr(N, "TEST_FRONT_CAP", 40)  # main-kernel frontier overflows in many groups
    h0 = dg["h"].clone()
    monkeypatch.setattr(N, "SPLIT_PREDICT", False)
    nl_ref = find_neighbors(dg, tree, box, 0, n)
    nc_ref, h_ref = dg["nc"].clone(), dg["h"].clone()
    sets_ref = neighbor_lists_as_sets(nl_ref, nc_ref)
    queued = dg.nc_queued
    assert queued > 0
    monkeypatch.setattr(N, "SPLIT_PREDICT", True)
    N._PRED.clear()
    for k in range(2):
        dg["h"].copy_(h0)
        nl = find_neighbors(dg, tree, box, 0, n)
        assert torch.equal(dg["nc"], nc_ref) and torch.equal(dg["h"], h_ref)
        assert neighbor_lists_as_sets(nl, dg["nc"]) == sets_ref
        # first search: nothing predicted; second: the main kernel skipped the recorded groups
        assert dg.nc_queued == queued if k == 0 else dg.nc_queued <= queued // 4


@pytest.mark.parametrize("hook", ["front", "caps"])
def test_gravity_spill_path(gpu, monkeypatch, hook):
    """groups overflowing the LDS stack (front) or the interaction-list slabs (caps) are evaluated by the fused
    global-stack kernel: same interactions, results equal to fp32 summation-order differences"""
    from sphexa_amd.ops import gravity as G
    from test_gravity import _setup as gsetup

    n = 20000
    box, ot, x, y, z, m, h = gsetup(n, gpu)
    c, mp = G.upsweep(ot, x, y, z, m, box, 0.5)
    acc = [torch.zeros(n, dtype=torch.float32, device=gpu) for _ in range(3)]
    st_ref = {}
    e_ref = G.compute_gravity(ot, c, mp, 0, n, x, y, z, h, m, 1.0, *acc, stats=st_ref)
    if hook == "front":
        monkeypatch.setattr(G, "TEST_FRONT_CAP", 16)
    else:
        monkeypatch.setattr(G, "TEST_CAPS", (256, 64))
    acc2 = [torch.zeros(n, dtype=torch.float32, device=gpu) for _ in range(3)]
    st = {}
    e2 = G.compute_gravity(ot, c, mp, 0, n, x, y, z, h, m, 1.0, *acc2, stats=st)
    assert st["fallback"] > st_ref["fallback"]
    assert st["p2p"] == st_ref["p2p"] and st["m2p"] == st_ref["m2p"]
    for a, b in zip(acc, acc2):
        assert float((a - b).abs().max()) < 1e-4 * float(a.abs().max())
    assert abs(e2 - e_ref) < 1e-5 * abs(e_ref)


def test_ve_step_nonuniform_mass_matches_cpu(gpu):
    """Masses with a 10 % spread: the GPU Gradh loop takes the stored-mass record path (SrcPos) instead of the
    uniform-mass fixed-point one (SrcXmQ); every other loop runs on fixed-point records either way."""
    results = {}
    for dev in ("cpu", gpu):
        d = P.ParticlesData(dev)
        prop = HydroVeProp(None, 0)
        prop.activate_fields(d)
        box = SedovGrid().init(0, 1, 14, d)
        g = torch.Generator().manual_seed(3)
        d["m"] = (d["m"].cpu() * (1 + 0.1 * torch.rand(d.size, generator=g))).to(d["m"].dtype).to(dev)
        if str(dev) != "cpu":
            assert H.uniform_mass(d) == 0.0
        dom = Domain(Comm(), box)
        prop.sync(dom, d)
        prop.step(dom, d)
        results[str(dev)] = {f: d[f].clone().cpu() for f in ("kx", "xm", "c11", "alpha", "ax", "du")}
    c, g = results["cpu"], results[str(gpu)]
    for f in ("kx", "xm", "c11", "alpha"):
        assert _rel(g[f], c[f]) < 2e-5, f
    _check(g, c, ("ax", "du"), 2e-5)


def test_uniform_mass_detection(gpu):
    d, prop, dom = _setup(gpu, n=8)
    m0 = float(d["m"][0])
    assert H.uniform_mass(d) == pytest.approx(m0)
    d["m"][3] *= 2  # in-place change bumps the tensor version: the cached value is not reused
    assert H.uniform_mass(d) == 0.0


def test_ve_step_fp64_records_matches_cpu(gpu, monkeypatch):
    """fp64-coordinate record path of the GPU pair loops (taken when the fixed-point quantum is too coarse for the
    smallest h, ops/hydro.py: fixed_point_code)"""
    monkeypatch.setattr(H, "fixed_point_code", lambda d, box: 0)
    results = {}
    for dev in ("cpu", gpu):
        d = P.ParticlesData(dev)
        prop = HydroVeProp(None, 0)
        prop.activate_fields(d)
        box = SedovGrid().init(0, 1, 14, d)
        dom = Domain(Comm(), box)
        prop.sync(dom, d)
        prop.step(dom, d)
        if str(dev) != "cpu":
            assert d.fixedPoint == 0
        results[str(dev)] = {f: d[f].clone().cpu() for f in ("kx", "xm", "c11", "alpha", "ax", "du")}
    c, g = results["cpu"], results[str(gpu)]
    for f in ("kx", "xm", "c11", "alpha"):
        assert _rel(g[f], c[f]) < 2e-5, f
    _check(g, c, ("ax", "du"), 2e-5)



def test_packed_list_overflow_rows_and_repeat(gpu, monkeypatch):
    """packed lists with 1 home row per group: every other row comes from the overflow stripes, and a first attempt
    with 8 rows per stripe runs out, so the search repeats with a larger pool; lists and the VE loops must not change
    (ops/neighbors.py _pool_plan, neighbors.hip encodeGroup)"""
    from sphexa_amd.ops import neighbors as N

    dg, pg, domg = _setup(gpu, 16, jitter=0.01)
    pg.sync(domg, dg)
    nl_ref = find_neighbors(dg, domg.octree, domg.box, 0, dg.size)
    sets_ref = neighbor_lists_as_sets(nl_ref, dg["nc"])
    H.compute_xmass(dg, nl_ref, domg.box)
    xm_ref = dg["xm"].clone()
    monkeypatch.setattr(N, "_pool_plan", lambda prev, groups, ng0, stripes: (1, 8))
    nl = find_neighbors(dg, domg.octree, domg.box, 0, dg.size)
    groups = (dg.size + 63) // 64
    assert nl.rows_used > groups  # overflow rows were taken
    assert neighbor_lists_as_sets(nl, dg["nc"]) == sets_ref
    H.compute_xmass(dg, nl, domg.box)
    assert torch.equal(dg["xm"], xm_ref)


@pytest.mark.parametrize("n", [16, 24])
def test_ve_step_momentum_handoff_identical(gpu, monkeypatch, n):
    """the momentum records written by the IAD / AV epilogues (ops/hydro.py MOM_HANDOFF: SrcMomQ64 rows + SrcMomSide
    {rho, alpha}) equal the ones packMomQ64Kernel packs: the step's fields are bit-identical with and without the
    hand-off"""
    results = []
    for handoff in (False, True):
        monkeypatch.setattr(H, "MOM_HANDOFF", handoff)
        d = P.ParticlesData(gpu)
        prop = HydroVeProp(None, 0)
        prop.activate_fields(d)
        box = SedovGrid().init(0, 1, n, d)
        dom = Domain(Comm(), box)
        prop.sync(dom, d)
        for _ in range(3):
            prop.step(dom, d)
            d.iteration += 1
        assert H.mom_split(d, False), "the split momentum records are the path under test"
        results.append({f: d[f].clone().cpu() for f in ("x", "y", "z", "vx", "vy", "vz", "temp", "du", "ax", "ay",
                                                         "az", "alpha")})
    for f in results[0]:
        assert torch.equal(results[0][f], results[1][f]), f


@pytest.mark.parametrize("case", ["sedov", "evrard"])
def test_fused_update_matches_separate_passes(gpu, monkeypatch, case):
    """the end of a deferred GPU step in one pass (hydro.hip updateStepKernel: positions, energy, h and the
    conserved-quantity sums) against the three separate launches: fields bit-identical, conserved sums to fp64
    summation order"""
    from sphexa_amd.app.simulation import Simulation
    from sphexa_amd.models import propagators as PR

    out = []
    for fused in (False, True):
        monkeypatch.setattr(PR, "FUSED_UPDATE", fused)
        sim = Simulation(case, n=20, prop="ve", device=gpu)
        sim.propagator.defer_host = True
        sim.run(3)
        sim.propagator.finish_host(sim.d)
        d = sim.d
        out.append(({f: sim.local(f).clone().cpu() for f in ("x", "y", "z", "vx", "vy", "vz", "h", "temp")},
                    (d.ecin, d.eint, d.egrav, d.linmom, d.angmom, d.totalNeighbors)))
    (fa, ca), (fb, cb) = out
    for f in fa:
        assert torch.equal(fa[f], fb[f]), f
    assert ca[5] == cb[5]
    for a, b in zip(ca[:5], cb[:5]):
        assert math.isclose(a, b, rel_tol=1e-12, abs_tol=1e-14), (ca, cb)


def test_fused_eos_identical(gpu, monkeypatch):
    """the VE EOS in the Gradh loop's epilogue (hydro.hip veDefGradhKernel, EosOut) equals the separate eosVeKernel:
    fields after three steps bit-identical"""
    from sphexa_amd.models import propagators as PR

    out = []
    for fused in (False, True):
        monkeypatch.setattr(PR, "FUSED_EOS", fused)
        d = P.ParticlesData(gpu)
        prop = HydroVeProp(None, 0)
        prop.activate_fields(d)
        box = SedovGrid().init(0, 1, 20, d)
        dom = Domain(Comm(), box)
        prop.sync(dom, d)
        for _ in range(3):
            prop.step(dom, d)
            d.iteration += 1
        out.append({f: d[f].clone().cpu() for f in ("x", "vx", "temp", "c", "prho", "du", "ax")})
    for f in out[0]:
        assert torch.equal(out[0][f], out[1][f]), f


def test_pair_loop_instances_agree(gpu):
    """the pair loops' specialized instances equal the generic ones after three Sedov steps: the momentum gathers as
    32-bit buffer loads (MomSplitLoaderT) bit for bit; the sinc^6 kernel function fixed at compile time (hydro.hip
    withKf) to rounding (the same products, but the compiler contracts the inlined constant forms into FMAs
    differently: 1-ulp differences in kx and the IAD coefficients at step 1)"""
    from sphexa_amd.ops import _lib

    fields = ("x", "vx", "temp", "c", "prho", "du", "ax", "alpha", "h")

    def run(kernel_fixed, mom_buf):
        _lib.hip().set_pair_paths(kernel_fixed=kernel_fixed, mom_buf=mom_buf)
        d = P.ParticlesData(gpu)
        prop = HydroVeProp(None, 0)
        prop.activate_fields(d)
        box = SedovGrid().init(0, 1, 20, d)
        dom = Domain(Comm(), box)
        prop.sync(dom, d)
        for _ in range(3):
            prop.step(dom, d)
            d.iteration += 1
        return {f: d[f].clone().cpu().double() for f in fields}

    try:
        generic = run(False, False)
        buf = run(False, True)
        fixed = run(True, True)
    finally:
        _lib.hip().set_pair_paths(kernel_fixed=True, mom_buf=True)
    for f in fields:
        assert torch.equal(buf[f], generic[f]), f
        scale = float(generic[f].abs().max())
        assert float((fixed[f] - generic[f]).abs().max()) <= 1e-5 * scale, f


def test_hilbert_table_keys(gpu):
    """the GPU key kernel's table walk equals the bit-serial hilbertKey kernel on 4 M random points (open and
    periodic boxes, points on the box faces included)"""
    from sphexa_amd.ops import _lib

    n = 4_000_000
    g = torch.Generator().manual_seed(5)
    for box in (Box.cube(-1.0, 2.0, OPEN), Box([0.0, -0.5, 0.25], [1.0, 0.7, 0.6], [PERIODIC] * 3)):
        lo, hi = torch.tensor(box.lo, dtype=torch.float64), torch.tensor(box.hi, dtype=torch.float64)
        p = lo + torch.rand(n, 3, generator=g, dtype=torch.float64) * (hi - lo)
        p[:1000] = lo
        p[1000:2000] = hi
        x, y, z = (p[:, k].contiguous().to(gpu) for k in range(3))
        a = torch.empty(n, dtype=torch.int64, device=gpu)
        b = torch.empty(n, dtype=torch.int64, device=gpu)
        s = _lib.stream()
        _lib.hip().compute_keys(n, x.data_ptr(), y.data_ptr(), z.data_ptr(), box.to_array(), sfc.HILBERT,
                                a.data_ptr(), s)
        _lib.hip().compute_keys_serial(n, x.data_ptr(), y.data_ptr(), z.data_ptr(), box.to_array(), sfc.HILBERT,
                                       b.data_ptr(), s)
        assert torch.equal(a, b)
    assert _lib.hip().hilbert_table_states() == 24
