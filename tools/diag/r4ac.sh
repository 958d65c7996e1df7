#!/bin/bash
# WGRAD split count target (WGRAD_WANT workgroups) on the BiSeNet and DeepLab steps + pw/pooled tests
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -k "pw_backward or pooled or arm or attention" > gpurun_out/r4ac_pytest.log 2>&1
o=gpurun_out/r4ac_ab.txt
: > $o
for r in 1 2; do
for lib in librtsds_hip var_ww384 var_ww768 var_ww1024; do
  for wl in bisenet-seg deeplab-seg; do
    RTSDS_LIB=$PWD/rtsds_amd/$lib.so timeout -k 10 300 python3 bench.py --workload $wl --no-cpu-baseline --no-infer --no-conv-profile > /tmp/r4ac.json 2>/dev/null
    python3 -c "import json,sys; d=json.load(open('/tmp/r4ac.json')); print('$lib', '$wl', d['value'], d['ms_per_step'])" >> $o
  done
done
done
echo ok
