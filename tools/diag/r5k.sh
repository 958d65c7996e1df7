#!/bin/bash
# kernel-level times of the layer1 weight gradient: direct kernel + reduce (base) vs GEMM (head)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in base head; do
  lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
  RTSDS_LIB=$PWD/$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r5k_$v -o run -- python3 tools/bench_conv.py 8 64 128 256 64 3 1 1 30 > gpurun_out/r5k_$v.log 2>&1 || exit 1
  python3 tools/kstats.py $(ls /tmp/r5k_$v/run_kernel_stats.csv) 33 > gpurun_out/r5k_$v.txt
done
