"""Global coordinate box with per-dimension boundary types.

Parity: reference domain/include/cstone/sfc/box.hpp:97-190 (Box, BoundaryType {open, periodic, fixed}, IO of the
"box" and "boundaryType" step attributes, box.hpp:168-175) and sfc/box_mpi.hpp:83-118 (makeGlobalBox: extrema of
non-periodic dimensions reduced over ranks every step).
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import List

OPEN, PERIODIC, FIXED = 0, 1, 2
_BC_CHARS = {OPEN: 0, PERIODIC: 1, FIXED: 2}


@dataclass
class Box:
    lo: List[float]
    hi: List[float]
    bc: List[int] = field(default_factory=lambda: [OPEN, OPEN, OPEN])

    @staticmethod
    def cube(lo: float, hi: float, bc: int = OPEN) -> "Box":
        return Box([lo] * 3, [hi] * 3, [bc] * 3)

    def lengths(self):
        return [self.hi[d] - self.lo[d] for d in range(3)]

    def to_array(self) -> List[float]:
        return [float(v) for v in self.lo] + [float(v) for v in self.hi] + [float(b) for b in self.bc]

    def any_periodic(self) -> bool:
        return PERIODIC in self.bc

    def attributes(self):
        """the reference stores box = [xmin, xmax, ymin, ymax, zmin, zmax] and boundaryType as 3 chars"""
        return {"box": [self.lo[0], self.hi[0], self.lo[1], self.hi[1], self.lo[2], self.hi[2]],
                "boundaryType": list(self.bc)}

    @staticmethod
    def from_attributes(box, bc) -> "Box":
        return Box([box[0], box[2], box[4]], [box[1], box[3], box[5]], [int(b) for b in bc])

    def copy(self) -> "Box":
        return Box(list(self.lo), list(self.hi), list(self.bc))
