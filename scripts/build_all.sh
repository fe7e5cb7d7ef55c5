#!/bin/bash
# every in-tree native module: OpenMP, HDF5 I/O, golden loops, gfx950 HIP and its device-check variant
set -e -o pipefail
cd "$(dirname "$0")/.."
python -m sphexa_amd.build_native | tail -1
python -m sphexa_amd.build_native --dcheck | tail -1
