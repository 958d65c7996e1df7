#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/bench_all.sh r4v bisenet-da deeplab-seg deeplab-da > gpurun_out/r4v_all.txt 2>&1
echo ok
