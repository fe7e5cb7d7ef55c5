"""Runs under SPHX_DEVICE_CHECKS=1 (device-check HIP build) for tests/test_gpu_guards.py: clean Sedov/Evrard steps
must report no failed check; a corrupted neighbor list must be reported (bit 0) without faulting the GPU."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from sphexa_amd.app.simulation import Simulation  # noqa: E402
from sphexa_amd.ops import _lib  # noqa: E402
from sphexa_amd.ops import hydro as H  # noqa: E402
from sphexa_amd.ops import neighbors as N  # noqa: E402


def main(mode: str):
    assert os.environ.get("SPHX_DEVICE_CHECKS") == "1"
    dev = torch.device("cuda", 0)
    if mode == "clean":
        Simulation("sedov", n=20, prop="ve", device=dev, out=None, quiet=True).run(2)
        Simulation("evrard", n=20, prop="ve", device=dev, out=None, quiet=True).run(1)
        assert _lib.hip().device_checks_enabled()
        print("clean ok", flush=True)
        return
    sim = Simulation("sedov", n=16, prop="ve", device=dev, out=None, quiet=True).run(1)
    d, nl = sim.d, sim.propagator.nl
    groups = (nl.last - nl.first + 63) // 64
    region = N.packed_table_region(groups, nl.ngmax)
    nl.nidx[region:] = 0x7FFF7FFF  # every slot: emit, step +16383 -> indices far past the particle count
    H.compute_xmass(d, nl, sim.domain.box)
    try:
        _lib.raise_on_device_check("corrupted list")
    except _lib.DeviceCheckError as e:
        torch.cuda.synchronize()
        print("caught:", e, flush=True)
        return
    raise SystemExit("corrupted neighbor list was not reported")


if __name__ == "__main__":
    main(sys.argv[1])
