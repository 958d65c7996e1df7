#!/bin/bash
# bilinear backward 4-tap load batching: parity, kernel times (base vs oldbilbwd), step A/B
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "bilinear" > gpurun_out/r6k_tests.txt 2>&1 || exit 1
for v in base oldbilbwd; do
  lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
  RTSDS_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6k_prof_$v -o run -- python3 bench.py --no-cpu-baseline --no-conv-profile --steps 10 --warmup 3 > gpurun_out/r6k_bench_$v.json 2>/dev/null || exit 1
done
timeout -k 10 900 bash tools/ab_step.sh 3 base oldbilbwd > gpurun_out/r6k_step.txt 2>&1
