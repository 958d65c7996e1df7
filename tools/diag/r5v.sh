#!/bin/bash
# BatchNorm-apply-on-load cost probe: the FWD implicit GEMM with y = bf16(max(x*sc+sh, 0)) applied
# to every A fragment after the ds_read (var_bnf.so, timing only) vs the plain kernel
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r5v_bnfold.txt; : > $o
for a in "8 128 64 128 128 3 1 1 30" "8 256 32 64 256 3 1 1 30" "8 512 16 32 512 3 1 1 30" "8 128 128 256 128 1 1 0 30"; do
  for v in base bnf base bnf; do
    lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
    echo "== $v $a" >> $o
    RTSDS_LIB=$PWD/$lib timeout -k 5 60 python3 tools/bench_conv.py $a 2>&1 | grep fwd >> $o || exit 1
  done
done
