#!/bin/bash
# A/B of LDS-DMA staging (RTSDS_CONV_GLDS=0 vs default) on the BiSeNet conv shapes
cd "$GRAFT_REPO_ROOT"
for shape in "${@:-8 128 64 128 128 3 1 1}"; do
  echo "== $shape"
  RTSDS_CONV_GLDS=0 timeout -k 10 120 python3 tools/bench_conv.py $shape 20 2>/dev/null | sed 's/^/  reg  /'
  timeout -k 10 120 python3 tools/bench_conv.py $shape 20 2>/dev/null | sed 's/^/  glds /'
done
