#!/bin/bash
# Conv micro-benchmarks (tools/bench_conv.py) against the diagnostic variants of
# tools/variants/conv_diag_variant.py: run_conv_diag.sh [variants...]
cd "$GRAFT_REPO_ROOT"
vars=${*:-"base nogather noepi both"}
while read -r a; do
  [ -z "$a" ] && continue
  echo "== $a"
  for v in $vars; do
    lib=rtsds_amd/var_diag_$v.so; [ -f rtsds_amd/var_$v.so ] && lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
    RTSDS_LIB=$PWD/$lib timeout -k 5 60 python3 tools/bench_conv.py $a | sed "s/^/  $v  /" || exit 1
  done
done <<'LIST'
8 128 64 128 128 3 1 1 30
8 64 256 512 128 3 2 1 30
8 128 128 256 256 3 2 1 30
8 256 32 64 256 3 1 1 30
8 512 16 32 512 3 1 1 30
8 64 128 256 64 3 1 1 30
8 128 64 128 128 1 1 0 30
8 512 64 128 128 1 1 0 30
8 2048 64 128 128 1 1 0 30
LIST
