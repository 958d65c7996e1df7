#!/bin/bash
# A/B of the LDS-DMA ring depth for the narrow (N <= 64) FWD / DGRAD tiles: ab_ring.sh LIB...
cd "$GRAFT_REPO_ROOT"
for lib in "$@"; do
  for shape in "8 64 128 256 64 3 1 1 30" "8 512 16 32 512 3 1 1 30" "8 256 32 64 256 3 1 1 30" "8 128 64 128 128 3 1 1 30" "4 1024 65 129 256 1 1 0 20" "4 64 129 257 64 3 1 1 20"; do
    echo "== $lib: $shape"
    RTSDS_LIB=$lib timeout -k 5 60 python3 tools/bench_conv.py $shape 2>/dev/null || exit 1
  done
done
