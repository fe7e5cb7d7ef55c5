"""Glass template blocks.

The reference reads a glass block (x, y, z in the unit cube) from an H5Part file given with ``--glass``
(init/utils.hpp readTemplateBlock). Without a file we use the built-in deterministic relaxed template
(base.make_glass_block), so every test case runs from generated initial conditions only.
"""

from __future__ import annotations

import numpy as np

from .base import glass_block


def load_block(path: str | None = None, n_side: int = 16) -> np.ndarray:
    if path:
        from ...utils import io as sio

        x, y, z = sio.read_template_block(path)
        X = np.stack([x, y, z], axis=1)
        return X
    return glass_block(n_side)
