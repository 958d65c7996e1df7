#!/bin/bash
# Whole-step + inference A/B on one box, variants interleaved: ab_step.sh ROUNDS base v1 v2 ...
# (base = rtsds_amd/librtsds_hip.so, vX = rtsds_amd/var_vX.so).  Prints per run:
# variant, train img/s, ms/step, inference FPS bs 8, bs 1.
cd "$GRAFT_REPO_ROOT"
rounds=$1; shift
for r in $(seq 1 $rounds); do
  for v in "$@"; do
    lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
    RTSDS_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-conv-profile > gpurun_out/ab_$v.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(sys.argv[2], d['value'], d['ms_per_step'], d.get('inference_fps_bs8'), d.get('inference_fps_bs1'), flush=True)" gpurun_out/ab_$v.json $v
  done
done
