#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r4ak_upce_final.txt
: > $o
for lib in var_head librtsds_hip; do
  RTSDS_LIB=$PWD/rtsds_amd/$lib.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r4ak_$lib -o run -- python3 tools/bench_upce.py 30 > /dev/null 2>&1
  python3 - /tmp/r4ak_$lib/run_kernel_stats.csv $lib >> $o <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "upce" in r["Name"]:
        print(sys.argv[2], r["Name"][:40], f"{float(r['AverageNs'])/1e3:.1f} us")
PY
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4ak_pytest.log 2>&1

o=gpurun_out/r4ak_ab.txt
: > $o
for r in 1 2; do
  for lib in var_head librtsds_hip; do
    RTSDS_LIB=$PWD/rtsds_amd/$lib.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-infer --no-conv-profile > /tmp/r4ak.json 2>/dev/null
    python3 -c "import json; d=json.load(open('/tmp/r4ak.json')); print('$lib', d['value'], d['ms_per_step'])" >> $o
  done
done
echo ok
