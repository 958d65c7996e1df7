#!/bin/bash
# narrow 1x1 weight gradient (pw.hip) vs HEAD's split-K GEMM path + suite + bench
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r4ab_diag.txt
: > $o
for r in 1 2; do
for lib in var_head librtsds_hip; do
  for a in "wgrad 8 19 64 128 19 1 1 0" "wgrad 8 256 32 64 19 1 1 0" "wgrad 8 512 16 32 19 1 1 0" "dgrad 8 512 1 1 512 1 1 0" "dgrad 8 256 1 1 256 1 1 0"; do
    RTSDS_LIB=$PWD/rtsds_amd/$lib.so timeout -k 5 60 python3 tools/diag/time_one.py $a >> $o 2>&1
  done
done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4ab_pytest.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r4ab_bench.json 2> gpurun_out/r4ab_bench.err
echo ok
