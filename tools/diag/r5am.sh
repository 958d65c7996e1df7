#!/bin/bash
# Epilogue cost probe: the bf16 LDS staging writes skipped (var_nost.so, timing only, wrong outputs)
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r5am_conv.txt; : > $o
for a in "8 128 64 128 128 3 1 1 30" "8 64 256 512 128 3 2 1 30" "8 128 128 256 256 3 2 1 30" "8 256 64 128 256 1 1 0 30"; do
  for v in base nost; do
    lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
    echo "== $v" >> $o
    RTSDS_LIB=$PWD/$lib timeout -k 5 60 python3 tools/bench_conv.py $a 2>&1 | grep -E "fwd|dgrad" >> $o || exit 1
  done
done
