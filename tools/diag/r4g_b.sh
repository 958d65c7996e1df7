#!/bin/bash
# round-4 evidence, part B: the other workloads' bench lines and profiles
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/bench_all.sh r4g bisenet-da deeplab-seg deeplab-da > gpurun_out/r4g_bench_all.txt 2>&1
bash tools/profile_all.sh r4g bisenet-da deeplab-seg deeplab-da
echo ok
