#!/bin/bash
# Representative conv layers (BiSeNet-R18 bs8 1024x512, DeepLabV2 bs4 1024x512) through
# tools/bench_conv.py, optionally against an alternative library: conv_suite.sh [LIB]
cd "$GRAFT_REPO_ROOT"
[ -n "$1" ] && export RTSDS_LIB=$1
while read -r a; do
  [ -z "$a" ] && continue
  timeout -k 5 60 python3 tools/bench_conv.py $a || exit 1
done <<'LIST'
8 64 128 256 64 3 1 1 30
8 64 128 256 128 3 2 1 30
8 128 64 128 128 3 1 1 30
8 128 64 128 256 3 2 1 30
8 256 32 64 256 3 1 1 30
8 256 16 32 512 3 1 1 30
8 512 16 32 512 3 1 1 30
4 64 129 257 256 1 1 0 20
4 256 129 257 64 1 1 0 20
4 1024 65 129 256 1 1 0 20
4 256 65 129 1024 1 1 0 20
4 256 65 129 256 3 1 2 20 2
4 512 65 129 512 3 1 4 20 4
4 2048 65 129 512 1 1 0 20
LIST
