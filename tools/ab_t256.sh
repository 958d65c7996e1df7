#!/bin/bash
# A/B of the 256x64 FWD tile on the BiSeNet 64-channel-output convs: ab_t256.sh LIB...
cd "$GRAFT_REPO_ROOT"
for lib in "$@"; do
  for shape in "8 3 512 1024 64 7 2 3 30" "8 3 512 1024 64 3 2 1 30" "8 64 128 256 64 3 1 1 30"; do
    echo "== $lib: $shape"
    RTSDS_LIB=$lib timeout -k 5 60 python3 tools/bench_conv.py $shape 2>/dev/null | grep fwd || exit 1
  done
  RTSDS_LIB=$lib timeout -k 10 200 python3 -u bench.py --steps 200 --no-cpu-baseline --no-infer --no-conv-profile 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print('bench', d['value'], d['ms_per_step'])" || exit 1
done
