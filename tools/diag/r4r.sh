#!/bin/bash
# hconv 8x32 tiles + Cout up to 512 (ResNet layer4): librtsds_hip vs var_k256 (layer4 on the GEMM)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r4r_diag.txt
: > $o
for r in 1 2; do
for lib in var_k256 librtsds_hip; do
  for a in "fwdstats 8 512 16 32 512 3 1 1" "eval 8 512 16 32 512 3 1 1" "dgrad 8 512 16 32 512 3 1 1" "fwdstats 8 256 32 64 256 3 1 1" "dgrad 8 256 32 64 256 3 1 1"; do
    RTSDS_LIB=$PWD/rtsds_amd/$lib.so timeout -k 5 60 python3 tools/diag/time_one.py $a >> $o 2>&1
  done
done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4r_pytest.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r4r_bench.json 2> gpurun_out/r4r_bench.err
echo ok
