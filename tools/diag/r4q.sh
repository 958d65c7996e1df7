#!/bin/bash
# hconv compile-time activation (var_head = HEAD) and 128x64 tiles for ResNet layer4 (var_m128)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r4q_diag.txt
: > $o
for r in 1 2; do
for lib in var_head librtsds_hip var_m128; do
  for a in "fwdstats 8 256 32 64 256 3 1 1" "eval 8 256 32 64 256 3 1 1" "dgrad 8 256 32 64 256 3 1 1" \
           "fwdstats 8 512 16 32 512 3 1 1" "eval 8 512 16 32 512 3 1 1" "dgrad 8 512 16 32 512 3 1 1" \
           "eval 8 1024 64 128 19 3 1 1" "fwdstats 8 256 32 64 512 3 2 1" "eval 8 256 32 64 512 3 2 1"; do
    RTSDS_LIB=$PWD/rtsds_amd/$lib.so timeout -k 5 60 python3 tools/diag/time_one.py $a >> $o 2>&1
  done
done
done
echo ok
