#!/bin/bash
# Whole-step A/B of a class-attribute toggle on one box (tools/ab_py.py): ab_py_attr.sh ROUNDS [ATTR=VALUE]
# default: FeatureFusionModule.fused_attention.  Prints per run: variant, img/s, ms/step, FPS bs 8, bs 1.
cd "$GRAFT_REPO_ROOT"
rounds=$1
attr=${2:-rtsds_amd.models.bisenet.build_bisenet.FeatureFusionModule.fused_attention}
for r in $(seq 1 $rounds); do
  for v in True False; do
    timeout -k 10 300 python3 tools/ab_py.py "$attr=$v" -- --no-cpu-baseline --no-conv-profile > gpurun_out/abp_$v.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(sys.argv[2], d['value'], d['ms_per_step'], d.get('inference_fps_bs8'), d.get('inference_fps_bs1'), flush=True)" gpurun_out/abp_$v.json $v
  done
done
