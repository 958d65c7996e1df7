#!/bin/bash
# BN backward micro-benchmark per variant .so, with a kernel trace: ab_bn.sh base v1 ...
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
shapes=${SHAPES:-"262144,64 65536,128 16384,256 4096,512 65536,256"}
for v in "$@"; do
  lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
  for sh in $shapes; do
    RTSDS_LIB=$PWD/$lib timeout -k 10 60 python3 tools/bench_bn.py ${sh//,/ } 20 2>/dev/null | sed "s/^/$v  /"
  done
  RTSDS_LIB=$PWD/$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abbn_$v -o run -- python3 tools/bench_bn.py 262144 64 20 > /dev/null 2>&1
done
