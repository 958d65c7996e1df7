#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r4i_diag.txt
: > $o
for lib in librtsds_hip var_nomfmadmastore; do
  for a in "fwd 8 64 128 256 64 3 1 1" "dgrad 8 64 128 256 64 3 1 1"; do
    RTSDS_LIB=$PWD/rtsds_amd/$lib.so timeout -k 5 60 python3 tools/diag/time_one.py $a >> $o 2>&1
  done
done
timeout -k 10 600 python -u -m pytest tests/test_configs_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread -k "bench_conv_shapes" > gpurun_out/r4i_pytest.log 2>&1 || echo "pytest failed"
echo ok
