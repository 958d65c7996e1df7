#!/bin/bash
# Whole-step A/B of Python-level changes on one box: the tree vs an older revision's Python
# (unpacked here by: git archive REV rtsds_amd bench.py | tar -x -C _abtree) running on the
# tree's library.  usage: ab_tree.sh ROUNDS   -> per run: variant, img/s, ms/step, FPS bs 8, bs 1
cd "$GRAFT_REPO_ROOT"
rounds=$1
for r in $(seq 1 $rounds); do
  for v in tree old; do
    d=.; [ "$v" = old ] && d=_abtree
    (cd $d && RTSDS_LIB=$GRAFT_REPO_ROOT/rtsds_amd/librtsds_hip.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-conv-profile) > gpurun_out/abt_$v.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(sys.argv[2], d['value'], d['ms_per_step'], d.get('inference_fps_bs8'), d.get('inference_fps_bs1'), flush=True)" gpurun_out/abt_$v.json $v
  done
done
