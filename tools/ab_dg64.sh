#!/bin/bash
# A/B of 64x64 data-gradient tiles for <= 64 input channels on large grids (BiSeNet layer1):
# ab_dg64.sh LIB...
cd "$GRAFT_REPO_ROOT"
for lib in "$@"; do
  RTSDS_LIB=$lib timeout -k 5 60 python3 tools/bench_conv.py 8 64 128 256 64 3 1 1 30 2>/dev/null | grep dgrad || exit 1
  RTSDS_LIB=$lib timeout -k 10 200 python3 -u bench.py --steps 300 --no-cpu-baseline --no-infer --no-conv-profile 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print('bench', d['value'], d['ms_per_step'])" || exit 1
done
