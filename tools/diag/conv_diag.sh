#!/bin/bash
# Where does the implicit-GEMM conv's time go?  Runs tools/conv_suite.sh's BiSeNet shapes
# against diagnostic builds of conv.hip (timing only, wrong results): no MFMA / no operand DMA
# after the first K-tile / no epilogue / the one-barrier NBUF=2 ring.  Output: gpurun_out/$1.txt
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-conv_diag}.txt
: > $out
for v in librtsds_hip nomfma nodma noepi onebar; do
  lib=rtsds_amd/var_$v.so; [ $v = librtsds_hip ] && lib=rtsds_amd/librtsds_hip.so
  echo "== $v" | tee -a $out
  while read -r a; do
    [ -z "$a" ] && continue
    RTSDS_LIB=$PWD/$lib timeout -k 5 60 python3 tools/bench_conv.py $a >> $out 2>&1 || exit 1
  done <<'LIST'
8 64 128 256 64 3 1 1 30
8 64 128 256 128 3 2 1 30
8 128 64 128 128 3 1 1 30
8 128 64 128 256 3 2 1 30
8 256 32 64 256 3 1 1 30
8 512 16 32 512 3 1 1 30
4 256 65 129 256 3 1 2 20 2
4 1024 65 129 256 1 1 0 20
LIST
done
