#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r4g_tap.txt
: > $o
for lib in var_notap librtsds_hip; do
  echo "== $lib" >> $o
  for a in "8 64 128 256 64 3 1 1 30" "4 64 129 257 64 3 1 1 30" "2 64 181 321 64 3 1 1 30"; do
    RTSDS_LIB=$PWD/rtsds_amd/$lib.so timeout -k 5 60 python3 tools/bench_conv.py $a >> $o 2>&1
  done
done
timeout -k 10 900 python -u -m pytest tests/test_ops_gpu.py tests/test_configs_gpu.py tests/test_models_gpu.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r4g_pytest.log 2>&1 || echo "pytest failed"
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r4g_bench.json 2> gpurun_out/r4g_bench.err
echo ok
