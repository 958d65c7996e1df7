#!/bin/bash
# A/B of the narrow-output conv paths (FWD split-K, WGRAD split count) on the 19-class convs:
# DeepLab ASPP branches (2048 -> 19, d 6 / 24) and BiSeNet's FFM conv (1024 -> 19).
cd "$GRAFT_REPO_ROOT"
for lib in "$@"; do
  for shape in "4 2048 65 129 19 3 1 6 20 6" "4 2048 65 129 19 3 1 24 20 24" "8 1024 64 128 19 3 1 1 20"; do
    echo "== $lib: $shape"
    RTSDS_LIB=$lib timeout -k 5 60 python3 tools/bench_conv.py $shape 2>/dev/null || exit 1
  done
done
