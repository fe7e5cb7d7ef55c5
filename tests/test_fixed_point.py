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
    d = _D(torch.full((4,), 1e-3, dtype=torch.float32))
    assert H.fixed_point_ok(d, Box([0.0] * 3, [1.0] * 3, [PERIODIC] * 3))
    assert H.fixed_point_ok(d, Box([0.0] * 3, [1.0] * 3, [OPEN] * 3))
    # open box 1000x larger: quantum 1e3 / 2^30 ~ 9e-7 > 2^-18 * 1e-3
    assert not H.fixed_point_ok(d, Box([0.0] * 3, [1e3] * 3, [OPEN] * 3))
    # periodic dimensions use the full 2^32 range
    assert H.fixed_point_ok(d, Box([0.0] * 3, [2.0] * 3, [PERIODIC] * 3))


def test_fixed_point_guard_tracks_h_updates():
    h = torch.full((4,), 1e-3, dtype=torch.float32)
    d = _D(h)
    box = Box([0.0] * 3, [1.0] * 3, [OPEN] * 3)
    assert H.fixed_point_ok(d, box)
    h[2] = 1e-9  # in-place update bumps the version: the cached minimum is recomputed
    assert not H.fixed_point_ok(d, box)
