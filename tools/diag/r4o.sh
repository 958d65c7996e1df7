#!/bin/bash
# templated-activation image convs: A/B vs HEAD (var_head) + their tests
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r4o_diag.txt
: > $o
for r in 1 2; do
for lib in var_head librtsds_hip; do
  for a in "fwdstats 8 3 512 1024 64 7 2 3" "eval 8 3 512 1024 64 7 2 3" "pool 8 3 512 1024 64 7 2 3" "fwdstats 8 3 512 1024 64 3 2 1" "eval 8 3 512 1024 64 3 2 1"; do
    RTSDS_LIB=$PWD/rtsds_amd/$lib.so timeout -k 5 60 python3 tools/diag/time_one.py $a >> $o 2>&1
  done
done
done
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -k "image_conv or stem or pool or bisenet" > gpurun_out/r4o_pytest.log 2>&1
echo ok
