#!/bin/bash
# can two RCCL ranks share the box's one GPU? (if so: 2-rank bench over RCCL)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/rccl; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 120 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 \
    scripts/probe_rccl_shared_gpu.py > $O/probe.log 2>&1; rc=$?
echo "probe rc $rc"; grep -v "^\s*$" $O/probe.log | tail -12
