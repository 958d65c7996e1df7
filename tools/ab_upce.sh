#!/bin/bash
# fused upsample+CE micro-benchmark per library variant: ab_upce.sh base v1 ...
cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
  RTSDS_LIB=$PWD/$lib timeout -k 10 120 python3 tools/bench_upce.py 30 2>/dev/null | sed "s/^/  $v  /"
done
