#!/bin/bash
# BatchNorm launch-shape variants (kernel-trace averages per kernel and shape)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/ab_bn2.sh base ra2048 ra4096 su4 rb1024 > gpurun_out/r4u_bn_bwd.txt 2>&1
BN_FWD=1 bash tools/ab_bn2.sh base ra2048 ra4096 > gpurun_out/r4u_bn_fwd.txt 2>&1
echo ok
