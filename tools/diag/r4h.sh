#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r4h_diag.txt
: > $o
for lib in librtsds_hip var_nodmastore var_nomfmadmastore var_notap; do
  for a in "fwd 8 64 128 256 64 3 1 1" "dgrad 8 64 128 256 64 3 1 1"; do
    RTSDS_LIB=$PWD/rtsds_amd/$lib.so timeout -k 5 60 python3 tools/diag/time_one.py $a >> $o 2>&1
  done
done
timeout -k 10 900 python -u -m pytest tests/test_ops_gpu.py tests/test_configs_gpu.py tests/test_models_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4h_pytest.log 2>&1 || echo "pytest failed"
echo ok
timeout -k 10 300 python -u tools/diag_copies.py > gpurun_out/r4h_copies.txt 2>&1 || echo "copies failed"
