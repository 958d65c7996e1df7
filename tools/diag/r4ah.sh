#!/bin/bash
# BN finalize tails with their per-channel operands loaded up front: kernel-trace A/B (HEAD = var_head)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export SHAPES="262144,64 65536,128 16384,256 4096,512 33540,1024"
bash tools/ab_bn2.sh head base > gpurun_out/r4ah_bn_bwd.txt 2>&1
BN_FWD=1 bash tools/ab_bn2.sh head base > gpurun_out/r4ah_bn_fwd.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4ah_pytest.log 2>&1
o=gpurun_out/r4ah_ab.txt
: > $o
for r in 1 2; do
  for lib in var_head librtsds_hip; do
    RTSDS_LIB=$PWD/rtsds_amd/$lib.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-infer --no-conv-profile > /tmp/r4ah.json 2>/dev/null
    python3 -c "import json; d=json.load(open('/tmp/r4ah.json')); print('$lib', d['value'], d['ms_per_step'])" >> $o
  done
done
echo ok
