#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export SHAPES="33540,256 33540,1024 33540,2048 132612,256 132612,64 33540,512"
bash tools/ab_bn2.sh base rb1024 rb2048 su4 > gpurun_out/r4z_bn_bwd.txt 2>&1
BN_Y=1 bash tools/ab_bn2.sh base rb1024 rb2048 su4 > gpurun_out/r4z_bn_bwd_y.txt 2>&1
echo ok
