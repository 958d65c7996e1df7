#!/bin/bash
# A/B of the tile for short-K GEMMs (K <= 512: DeepLab layer3 1x1 convs) : ab_shortk.sh LIB...
cd "$GRAFT_REPO_ROOT"
for lib in "$@"; do
  for shape in "4 1024 65 129 256 1 1 0 20" "4 256 65 129 1024 1 1 0 20" "4 64 129 257 256 1 1 0 20" "8 64 128 256 128 3 2 1 30"; do
    echo "== $lib: $shape"
    RTSDS_LIB=$lib timeout -k 5 60 python3 tools/bench_conv.py $shape 2>/dev/null || exit 1
  done
done
