#!/bin/bash
# Run the conv micro-benchmark for each variant .so given: ab_variants.sh base prio mid ...
cd "$GRAFT_REPO_ROOT"
shapes=${SHAPES:-"8,128,64,128,128,3,1,1 8,64,128,256,64,3,1,1 8,256,32,64,256,3,1,1 8,512,16,32,512,3,1,1"}
for sh in $shapes; do
  shape=${sh//,/ }
  echo "== $shape"
  for v in "$@"; do
    lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
    RTSDS_LIB=$PWD/$lib timeout -k 10 120 python3 tools/bench_conv.py $shape 20 2>/dev/null | sed "s/^/  $v  /"
  done
done
