#!/bin/bash
# A/B of WGRAD split counts on the DeepLab / BiSeNet wgrad shapes: ab_wgrad.sh LIB...
cd "$GRAFT_REPO_ROOT"
for lib in "$@"; do
  for shape in "4 512 65 129 512 3 1 4 20 4" "4 1024 65 129 2048 1 1 0 20" "4 2048 65 129 512 1 1 0 20" "8 64 128 256 64 3 1 1 30" "8 256 32 64 256 3 1 1 30" "8 512 16 32 512 3 1 1 30"; do
    echo "== $lib: $shape"
    RTSDS_LIB=$lib timeout -k 5 60 python3 tools/bench_conv.py $shape 2>/dev/null | grep wgrad || exit 1
  done
done
