#!/bin/bash
# Stream-priority probe: the "split" replay (per-lane segment graphs on their own streams) with
# the branch lanes at the highest stream priority (var_prio.so) vs split and branches (current).
cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  for v in "base branches" "base split" "prio split"; do
    set -- $v
    lib=rtsds_amd/var_$1.so; [ "$1" = base ] && lib=rtsds_amd/librtsds_hip.so
    RTSDS_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-conv-profile --no-infer --submit $2 > gpurun_out/r5ad_bench.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'])" gpurun_out/r5ad_bench.json $1 $2 | tee -a gpurun_out/r5ad_ab.txt
  done
done
