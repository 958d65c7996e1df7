#!/bin/bash
# A/B of the data-gradient tile for <= 32 input channels (TinyD conv1 on the channel-padded
# probabilities: 32 -> 64, 4x4 s2) : ab_dnarrow.sh LIB...
cd "$GRAFT_REPO_ROOT"
for lib in "$@"; do
  for shape in "8 32 512 1024 64 4 2 1 10" "2 32 720 1280 64 4 2 1 10"; do
    echo "== $lib: $shape"
    RTSDS_LIB=$lib timeout -k 5 60 python3 tools/bench_conv.py $shape 2>/dev/null || exit 1
  done
done
