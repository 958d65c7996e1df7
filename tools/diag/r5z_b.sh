#!/bin/bash
# round-5 (end of session) evidence, part B: the other workloads' bench lines, BiSeNet-DA profiles
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/bench_all.sh r5z bisenet-da deeplab-seg deeplab-da > gpurun_out/r5z_bench_all.txt 2>&1
bash tools/profile_all.sh r5z bisenet-da
echo ok
