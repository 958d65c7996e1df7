#!/bin/bash
cd "$GRAFT_REPO_ROOT"
[ -n "$1" ] && export RTSDS_LIB=$1
while read -r a; do
  [ -z "$a" ] && continue
  timeout -k 5 60 python3 tools/bench_conv_stats.py $a 2>/dev/null || exit 1
done <<'LIST'
8 64 128 256 64 3 1 1 30
8 128 64 128 128 3 1 1 30
8 256 32 64 256 3 1 1 30
8 512 16 32 512 3 1 1 30
8 64 128 256 128 1 2 0 30
4 256 65 129 1024 1 1 0 20
4 1024 65 129 256 1 1 0 20
4 256 65 129 256 3 1 2 20 2
4 64 129 257 256 1 1 0 20
LIST
