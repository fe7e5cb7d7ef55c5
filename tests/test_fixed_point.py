"""CPU tier: the switch between fixed-point and fp64-coordinate records of the GPU pair loops (ops/hydro.py)."""

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


def test_fixed_point_guard():
    d = _D(torch.full((4,), 4e-3, dtype=torch.float32))
    assert H.FIXED_POINT_REL_QUANTUM <= 2.0 ** -22
    assert H.fixed_point_ok(d, Box([0.0] * 3, [1.0] * 3, [PERIODIC] * 3))
    # open dimensions use 2^31 steps (the box is the particles' bounding box): 2 / 2^31 = 9.3e-10 <= 2^-22 * 4e-3
    assert H.fixed_point_ok(d, Box([0.0] * 3, [2.0] * 3, [OPEN] * 3))
    assert not H.fixed_point_ok(d, Box([0.0] * 3, [2.1] * 3, [OPEN] * 3))
    # periodic dimensions use the full 2^32 range
    assert H.fixed_point_ok(d, Box([0.0] * 3, [4.0] * 3, [PERIODIC] * 3))
    assert not H.fixed_point_ok(d, Box([0.0] * 3, [4.2] * 3, [PERIODIC] * 3))


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
