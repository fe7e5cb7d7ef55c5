#!/usr/bin/env python3
"""debug aid: device memory around the record workspace and field acquire/release calls of one VE step"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sphexa_amd.app.simulation import Simulation  # noqa: E402
from sphexa_amd.models import particles as P  # noqa: E402
from sphexa_amd.ops import hydro as H  # noqa: E402
from sphexa_amd.parallel.comm import init_distributed  # noqa: E402

comm = init_distributed("nccl")
sim = Simulation("sedov", n=100, prop="ve", device=torch.device("cuda", 0), comm=comm, out=None, quiet=True)
n = sim.d.numParticlesGlobal
sim.step()


def mb():
    return torch.cuda.memory_allocated() / n


orig_rec, orig_acq, orig_rel = H._rec, P.ParticlesData.acquire, P.ParticlesData.release


def rec(d, which=0, loop="mom"):
    a = mb()
    r = orig_rec(d, which, loop)
    print(f"_rec({which},{loop}) {a:.0f} -> {mb():.0f} B/p (peak {torch.cuda.max_memory_allocated() / n:.0f})")
    return r


def acq(self, *names):
    a = mb()
    orig_acq(self, *names)
    print(f"acquire{names} {a:.0f} -> {mb():.0f}")


def rel(self, *names):
    a = mb()
    orig_rel(self, *names)
    print(f"release{names} {a:.0f} -> {mb():.0f}")


H._rec, P.ParticlesData.acquire, P.ParticlesData.release = rec, acq, rel
torch.cuda.reset_peak_memory_stats()
sim.step()
print(f"end {mb():.0f} peak {torch.cuda.max_memory_allocated() / n:.0f}")
