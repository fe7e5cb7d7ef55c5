"""LDS-staged pair loops (csrc/hip/staged.h) against the per-lane-gather loops on the same inputs: every VE step field
after two steps of a case, fp32 summation-order tolerance (the staged loops add W partial sums per target).

The windowed path (a group's source union larger than the LDS capacity or spread over more than 63 chunk slots) is
forced with a neighbor count of ~300 (unions of ~2,000 sources)."""

import pytest
import torch

from sphexa_amd.app.simulation import Simulation
from sphexa_amd.ops import _lib

pytestmark = pytest.mark.gpu

FIELDS = ("x", "y", "z", "vx", "vy", "vz", "h", "temp", "u", "alpha", "xm", "kx", "du", "c", "nc")


def _run(gpu, case, n, mask, steps=2, ng=None):
    hp = _lib.hip()
    old = hp.staged_mask()
    hp.set_staged(mask)
    try:
        sim = Simulation(case, n=n, device=gpu)
        if ng is not None:
            # ~ng0 neighbors from the first search on: h scaled from the case's 100-neighbor value
            sim.d.ng0, sim.d.ngmax = ng
            sim.d["h"] = sim.d["h"] * (ng[0] / 100.0) ** (1.0 / 3.0)
        sim.run(steps)
        torch.cuda.synchronize()
        out = {}
        for f in FIELDS:
            try:
                v = sim.local(f)
            except Exception:  # (fields a case does not allocate)
                continue
            if v is not None and v.numel():
                out[f] = v.double().cpu()
        return out
    finally:
        hp.set_staged(old)


def _compare(a, b, tol):
    assert a.keys() == b.keys() and "x" in a
    worst = {}
    for f in a:
        scale = float(a[f].abs().max()) or 1.0
        err = float((a[f] - b[f]).abs().max()) / scale
        worst[f] = err
        assert torch.isfinite(b[f]).all(), f
    bad = {f: e for f, e in worst.items() if e > tol}
    assert not bad, f"staged vs gathered: {bad} (all: {worst})"


@pytest.mark.parametrize("case,n,mask", [("sedov", 24, 1), ("sedov", 24, 31), ("noh", 24, 31), ("evrard", 24, 31)])
def test_staged_loops_match_gathered(gpu, case, n, mask):
    a = _run(gpu, case, n, 0)
    b = _run(gpu, case, n, mask)
    _compare(a, b, 2e-5)


def test_staged_windows_match_gathered(gpu):
    """~300 neighbors per particle: most groups need several LDS windows"""
    a = _run(gpu, "sedov", 20, 0, steps=1, ng=(300, 400))
    b = _run(gpu, "sedov", 20, 31, steps=1, ng=(300, 400))
    assert float(a["nc"].mean()) > 250
    _compare(a, b, 2e-5)


def test_search_masks_cover_every_code(gpu):
    """the search's per-slot staged-source masks (packed_list.hpp; stored while a staged loop is enabled or
    set_list_masks) have the bit of every list entry: the union the staged loops copy into LDS holds every neighbor"""
    import numpy as np

    from sphexa_amd.ops.neighbors import GROUP, packed_table_ints, packed_table_region

    hp = _lib.hip()
    hp.set_list_masks(True)
    try:
        sim = Simulation("evrard", n=24, device=gpu)
        sim.run(1)
    finally:
        hp.set_list_masks(False)
    nl = sim.propagator.nl
    n = nl.last - nl.first
    G = (n + GROUP - 1) // GROUP
    buf = nl.nidx.cpu().numpy()
    Ti = packed_table_ints(nl.ngmax)
    tab = buf[:G * Ti].reshape(G, Ti)
    rows = buf[packed_table_region(G, nl.ngmax):].reshape(-1, 256)
    rows16 = rows.view(np.uint16).reshape(-1, 64, 8)
    checked = 0
    for g in range(0, G, max(1, G // 64)):
        nblk, w = int(tab[g, 0]), int(tab[g, 1])
        nch, tc, T = w & 0x3FF, (w >> 10) & 0x3F, w >> 16
        assert T >= tc + (nch + 127) // 128
        r = tab[g, 2:]
        masks = [int(np.uint32(rows[r[tc + s // 128], 2 * (s % 128)])) |
                 int(np.uint32(rows[r[tc + s // 128], 2 * (s % 128) + 1])) << 32 for s in range(nch)]
        codes = rows16[r[T:T + nblk]].reshape(-1)
        slot, k = codes & 0x3FF, codes >> 10
        real = slot > 0
        assert all((masks[s] >> kk) & 1 for s, kk in zip(slot[real].tolist(), k[real].tolist()))
        checked += int(real.sum())
    assert checked > 1000
