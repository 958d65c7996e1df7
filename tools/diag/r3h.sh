#!/bin/bash
# hcw (weight-stationary halo conv) correctness + speed
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_configs_gpu.py tests/test_ops_gpu.py -x -q --timeout 300 --timeout-method thread -k "conv" > $o/r3h_pytest.log 2>&1
for shape in "8 64 128 256 64 3 1 1 30" "4 64 129 257 64 3 1 1 20"; do
  timeout -k 5 60 python3 tools/bench_conv.py $shape >> $o/r3h_conv.txt 2>&1
done
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $o/r3h_bench.json 2> $o/r3h_bench.err
echo ok
