#!/bin/bash
# whole-step A/B: direct layer1 weight gradient (current) vs the split-K GEMM (35b2689 conv units)
cd "$GRAFT_REPO_ROOT"
for v in base notw base notw base notw; do
  lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
  RTSDS_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-conv-profile --no-infer > gpurun_out/r5q_bench_$v.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r5q_bench_$v.json $v | tee -a gpurun_out/r5q_ab.txt
done
