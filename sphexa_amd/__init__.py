"""sphexa_amd — an MI355X-native SPH + self-gravity engine with the capabilities of SPH-EXA.

Layout
  models/    particle container, propagators (ve, std, nbody, turbulence), initial conditions, observables, gravity
  ops/       native operator wrappers: SFC keys/sort, cornerstone octree, neighbor search, SPH loops, gravity
  parallel/  one-process-per-GPU communication (RCCL/gloo via torch.distributed) and SFC domain decomposition
  utils/     box, kernel tables, timers, argument parsing, H5Part/ASCII I/O
  app/       the ``sphexa`` command-line driver
  csrc/      C++/HIP sources of the native modules (_sphx_cpu, _sphx_hip, _sphx_io)
"""

__version__ = "0.1.0"
