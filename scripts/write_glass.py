#!/usr/bin/env python3
"""Write the built-in glass template block (models/init/base.glass_block) as an H5Part file with x, y, z in step 0,
the format the reference reads with --glass (main/src/init/utils.hpp readTemplateBlock). Used to give a locally
built reference binary the same Evrard / Noh glass initial conditions as ours (scripts/gpu_ref.sh).
usage: python scripts/write_glass.py OUT.h5 [n_side=16]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from sphexa_amd.models.init.base import glass_block  # noqa: E402
from sphexa_amd.utils.io import H5PartWriter  # noqa: E402


def main():
    out = sys.argv[1]
    n_side = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    X = glass_block(n_side)
    if os.path.exists(out):
        os.remove(out)
    w = H5PartWriter()
    w.add_step(0, X.shape[0], out)
    for k, c in enumerate("xyz"):
        w.write_field(c, np.ascontiguousarray(X[:, k], dtype=np.float64))
    w.close_step()
    print(f"wrote {X.shape[0]} glass particles to {out}")


if __name__ == "__main__":
    main()
