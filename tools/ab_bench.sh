#!/bin/bash
# Whole-step A/B: bench.py (train step only) per variant .so: ab_bench.sh base v1 v2 ...
cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
  RTSDS_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-infer > gpurun_out/ab_$v.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/ab_$v.json $v
done
