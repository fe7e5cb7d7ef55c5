"""CPU tier: the switch between fixed-point and fp64-coordinate records of the GPU pair loops (ops/hydro.py)."""

import numpy as np
import pytest
import torch

from sphexa_amd.ops import hydro as H
from sphexa_amd.utils.box import Box, OPEN, PERIODIC


class _D:
    def __init__(self, h):
        self._h = h
        self.size = h.numel()

    def __getitem__(self, name):
        assert name == "h"
        return self._h


def _shifts(code):
    return [(code >> (1 + 5 * k)) & 31 for k in range(3)]


def test_fixed_point_guard():
    d = _D(torch.full((4,), 4e-3, dtype=torch.float32))
    assert H.FIXED_POINT_REL_QUANTUM <= 2.0 ** -22
    assert H.fixed_point_ok(d, Box([0.0] * 3, [1.0] * 3, [PERIODIC] * 3))
    # the wrap period shrinks by powers of two while half of it exceeds 1.125 * 2 h_max = 9e-3, less one shift of
    # headroom: periodic L = 1 -> 1/16 (shift 4), open L = 1 -> 2/32 (shift 5), open L = 2.1 -> 4.2/64 (shift 6)
    fresh = lambda b: H.frame_code(b, 4e-3, 4e-3)  # noqa: E731
    assert _shifts(fresh(Box([0.0] * 3, [1.0] * 3, [PERIODIC] * 3))) == [4] * 3
    assert _shifts(fresh(Box([0.0] * 3, [1.0] * 3, [OPEN] * 3))) == [5] * 3
    assert _shifts(fresh(Box([0.0] * 3, [2.1] * 3, [OPEN] * 3))) == [6] * 3
    assert _shifts(fresh(Box([0.0, 0.0, 0.0], [1.0, 2.1, 0.5], [PERIODIC, OPEN, OPEN]))) == [4, 6, 4]
    # a valid previous code is kept (no flicker between steps); an invalid one is replaced
    b = Box([0.0] * 3, [1.0] * 3, [OPEN] * 3)
    c5 = fresh(b)
    assert H.frame_code(b, 4e-3, 1.3e-2, c5) == c5  # h_max grew within the headroom
    assert H.frame_code(b, 4e-3, 1.5e-2, c5) != c5 and H.frame_valid(b, H.frame_code(b, 4e-3, 1.5e-2, c5), 4e-3, 1.5e-2)
    assert all(not H.frame_valid(b, c5 + (2 << (1 + 5 * k)), 4e-3, 4e-3) for k in range(3))
    # boxes too small for an unambiguous wrap at shift 0 (an open pair at lo and hi would flip sign)
    assert H.frame_code(Box([0.0] * 3, [0.008] * 3, [OPEN] * 3), 4e-3, 4e-3) == 0
    assert H.frame_code(Box([0.0] * 3, [0.017] * 3, [PERIODIC] * 3), 4e-3, 4e-3) == 0
    # a small h_min against a large h_max: the quantum of the period that h_max needs is too coarse -> fp64
    assert H.frame_code(Box([0.0] * 3, [1.0] * 3, [OPEN] * 3), 1e-6, 1e-2) == 0
    assert H.frame_code(Box([0.0] * 3, [1.0] * 3, [OPEN] * 3), 1e-4, 1e-2) != 0


def _wrap_sep(code, box, xi, xj):
    """the GPU pair separation of two fixed-point records (sph_math.hpp quantize + pairSep), emulated in int64"""
    out = []
    for k, (lo, L, bc) in enumerate(zip(box.lo, box.lengths(), box.bc)):
        sh = (code >> (1 + 5 * k)) & 31
        sc = 2.0 ** ((32 if bc == PERIODIC else 31) + sh) / L
        oi = np.rint((xi[:, k] - lo) * sc).astype(np.int64) & 0xFFFFFFFF
        oj = np.rint((xj[:, k] - lo) * sc).astype(np.int64) & 0xFFFFFFFF
        d = (oi - oj) & 0xFFFFFFFF
        d = np.where(d >= 2 ** 31, d - 2 ** 32, d)
        out.append(d / sc)
    return np.stack(out, 1)


@pytest.mark.parametrize("bc", [OPEN, PERIODIC])
def test_shifted_frame_separations_are_exact_minimum_images(bc):
    """every pair within 2 h_max: the wrapped 32-bit difference in the shifted frame is the (minimum-image)
    separation up to one quantum per component, for pairs anywhere in the box, across the periodic seam included"""
    rng = np.random.default_rng(3)
    box = Box([-1.0, -0.5, 0.25], [1.0, 0.7, 0.6], [bc] * 3)
    hmax = 0.01
    code = H.frame_code(box, 2e-3, hmax)
    assert code != 0 and min(_shifts(code)) > 0
    n = 200000
    lo, L = np.array(box.lo), np.array(box.lengths())
    xi = lo + rng.random((n, 3)) * L
    dx = rng.normal(size=(n, 3))
    dx *= (2 * hmax * rng.random(n) ** (1 / 3) / np.linalg.norm(dx, axis=1))[:, None]
    xj = xi - dx
    if bc == PERIODIC:
        xj = lo + np.mod(xj - lo, L)  # sources wrapped into the box: the pair crosses the seam
    else:
        keep = np.all((xj >= lo) & (xj <= lo + L), axis=1)
        xi, xj, dx = xi[keep], xj[keep], dx[keep]
    sep = _wrap_sep(code, box, xi, xj)
    q = H.quantum(box, code)
    assert np.abs(sep - dx).max() <= 1.01 * q
    assert q <= H.FIXED_POINT_REL_QUANTUM * 2e-3


def test_fixed_point_guard_tracks_h_updates():
    h = torch.full((4,), 4e-3, dtype=torch.float32)
    d = _D(h)
    box = Box([0.0] * 3, [1.0] * 3, [OPEN] * 3)
    assert H.fixed_point_ok(d, box)
    h[2] = 1e-9  # in-place update bumps the version: the cached minimum is recomputed
    assert not H.fixed_point_ok(d, box)


def test_native_h_writers_invalidate_the_cache():
    """update_smoothing_length writes h through its data pointer (no version bump): the cached minimum must go"""
    from sphexa_amd.models import particles as P

    d = P.ParticlesData("cpu")
    d.set_conserved("x", "y", "z", "h", "m")
    d.set_dependent("nc")
    d.resize(64)
    d["h"] = 4e-3
    d["nc"] = 1  # far too few neighbors: update_h grows h
    box = Box([0.0] * 3, [1.0] * 3, [OPEN] * 3)
    assert H.fixed_point_ok(d, box)
    d._h_min_global = 1e-9  # a stale per-step value
    H.update_smoothing_length(d, 0, 64)
    assert getattr(d, "_h_min_global", None) is None
    assert H.fixed_point_ok(d, box)
    assert H.fixed_point_ok(d, box) and d._h_min[1] > 4e-3


def test_global_h_min_carries_the_uniform_mass():
    """set_global_h_min reduces h min and the mass extremes in one copy and primes uniform_mass's cache"""
    from sphexa_amd.models import particles as P

    d = P.ParticlesData("cpu")
    d.set_conserved("x", "y", "z", "h", "m")
    d.resize(32)
    d["h"] = torch.linspace(0.01, 0.02, 32, dtype=torch.float32)
    d["m"] = 0.5
    H.set_global_h_min(d, None)
    assert abs(d._h_min_global - 0.01) < 1e-9
    key, val = d._m_uniform
    assert val == 0.5 and key[0] == d["m"].data_ptr()
    assert H.uniform_mass(d) == 0.5
    d["m"][3] = 0.25  # in-place change bumps the version: recomputed, no longer uniform
    assert H.uniform_mass(d) == 0.0
    H.set_global_h_min(d, None)
    assert d._m_uniform[1] == 0.0
