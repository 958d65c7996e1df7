#!/bin/bash
# same-box A/B: attention-module gradient joins (working tree = HEAD) vs joins off (ab_prev2/)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r4ag_ab.txt
: > $o
for r in 1 2 3; do
  for v in ab_prev2/bench.py bench.py; do
    timeout -k 10 300 python3 $v --no-cpu-baseline --no-infer --no-conv-profile > /tmp/r4ag.json 2>/dev/null
    python3 -c "import json; d=json.load(open('/tmp/r4ag.json')); print('$v', d['value'], d['ms_per_step'])" >> $o
  done
done
echo ok
