#!/bin/bash
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ops_gpu.py -k "conv or hconv" \
  tests/test_configs_gpu.py::test_bench_conv_shapes > gpurun_out/r6c_pytest.log 2>&1 || { tail -30 gpurun_out/r6c_pytest.log; exit 1; }
tail -2 gpurun_out/r6c_pytest.log
for sh in "8 64 256 512 128 3 2 1" "8 128 128 256 256 3 2 1" "8 128 64 128 128 3 1 1" "8 256 32 64 256 3 1 1"; do
  for v in base r5; do
    lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
    RTSDS_LIB=$PWD/$lib timeout -k 5 60 python3 tools/bench_conv_stats.py $sh 30 2>/dev/null | sed "s/^/$v /"
  done
done > gpurun_out/r6c_stats.txt
timeout -k 10 600 bash tools/variants/run_conv_diag.sh base r5 > gpurun_out/r6c_conv.txt 2>&1
timeout -k 10 900 bash tools/ab_step.sh 2 base r5 > gpurun_out/r6c_step.txt 2>&1
