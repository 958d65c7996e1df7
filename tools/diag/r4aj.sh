#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4aj_pytest.log 2>&1
o=gpurun_out/r4aj_ab.txt
: > $o
for r in 1 2; do
  for lib in var_head librtsds_hip; do
    RTSDS_LIB=$PWD/rtsds_amd/$lib.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-infer --no-conv-profile > /tmp/r4aj.json 2>/dev/null
    python3 -c "import json; d=json.load(open('/tmp/r4aj.json')); print('$lib', d['value'], d['ms_per_step'])" >> $o
  done
done
echo ok
