#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r4j_diag.txt
: > $o
for lib in librtsds_hip var_notap; do
  for a in "fwd 8 64 128 256 64 3 1 1" "dgrad 8 64 128 256 64 3 1 1"; do
    RTSDS_LIB=$PWD/rtsds_amd/$lib.so timeout -k 5 60 python3 tools/diag/time_one.py $a >> $o 2>&1
  done
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4j_pytest.log 2>&1 || echo "pytest failed"
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r4j_bench.json 2> gpurun_out/r4j_bench.err
echo ok
