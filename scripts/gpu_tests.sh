#!/bin/bash
# GPU test pass used with gpurun: runs the gpu-marked tests given as arguments (default: all) in ONE process.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 ${GPU_TEST_TIMEOUT:-500} python -m pytest ${@:-tests} -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1
