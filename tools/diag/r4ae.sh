#!/bin/bash
# WGRAD grouped tile order (WGRAD_GROUP_M) vs M-fastest
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r4ae_ab.txt
: > $o
for r in 1 2; do
for lib in librtsds_hip var_wg2 var_wg4 var_wg8; do
  for wl in deeplab-seg bisenet-seg; do
    RTSDS_LIB=$PWD/rtsds_amd/$lib.so timeout -k 10 300 python3 bench.py --workload $wl --no-cpu-baseline --no-infer --no-conv-profile > /tmp/r4ae.json 2>/dev/null
    python3 -c "import json,sys; d=json.load(open('/tmp/r4ae.json')); print('$lib', '$wl', d['value'], d['ms_per_step'])" >> $o
  done
done
done
echo ok
