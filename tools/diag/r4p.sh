#!/bin/bash
# compile-time activation / epilogue variants (conv_gemm, tapconv, image convs): A/B vs HEAD
# (var_head) + the full GPU suite + bench
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r4p_diag.txt
: > $o
for r in 1 2; do
for lib in var_head librtsds_hip; do
  for a in "fwd 8 64 128 256 64 3 1 1" "fwdstats 8 64 128 256 64 3 1 1" "eval 8 64 128 256 64 3 1 1" "dgrad 8 64 128 256 64 3 1 1" \
           "fwdstats 8 128 64 128 128 3 1 1" "eval 8 128 64 128 128 3 1 1" "dgrad 8 128 64 128 128 3 1 1" \
           "fwdstats 8 256 32 64 256 3 1 1" "eval 8 256 32 64 256 3 1 1" "dgrad 8 256 32 64 256 3 1 1" \
           "fwdstats 8 512 16 32 512 3 1 1" "eval 8 512 16 32 512 3 1 1" "dgrad 8 512 16 32 512 3 1 1" \
           "fwdstats 8 64 256 512 128 3 2 1" "eval 8 64 256 512 128 3 2 1" \
           "fwdstats 8 3 512 1024 64 7 2 3" "eval 8 3 512 1024 64 7 2 3" "pool 8 3 512 1024 64 7 2 3" "eval 8 3 512 1024 64 3 2 1"; do
    RTSDS_LIB=$PWD/rtsds_amd/$lib.so timeout -k 5 60 python3 tools/diag/time_one.py $a >> $o 2>&1
  done
done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4p_pytest.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r4p_bench.json 2> gpurun_out/r4p_bench.err
echo ok
