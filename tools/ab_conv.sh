#!/bin/bash
# A/B of LDS-DMA staging on the mid-layer conv shapes (RTSDS_CONV_GLDS=0 vs default)
set -e
cd "$GRAFT_REPO_ROOT"
for shape in "8 128 64 128 128 3 1 1" "8 64 128 256 64 3 1 1" "8 256 32 64 256 3 1 1" "8 512 16 32 512 3 1 1" "8 128 64 128 256 3 2 1"; do
  echo "== $shape"
  RTSDS_CONV_GLDS=0 timeout -k 10 120 python3 tools/bench_conv.py $shape 20 2>/dev/null | sed 's/^/  reg  /'
  timeout -k 10 120 python3 tools/bench_conv.py $shape 20 2>/dev/null | sed 's/^/  glds /'
done
