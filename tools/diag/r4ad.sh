#!/bin/bash
# upce occupancy (4 waves / SIMD with spills) and 16-row tiles, kernel-trace averages
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r4ad_upce.txt
: > $o
for lib in librtsds_hip var_up4 var_up16; do
  RTSDS_LIB=$PWD/rtsds_amd/$lib.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r4ad_$lib -o run -- python3 tools/bench_upce.py 30 > /dev/null 2>&1
  python3 - /tmp/r4ad_$lib/run_kernel_stats.csv $lib >> $o <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "upce" in r["Name"]:
        print(sys.argv[2], r["Name"][:40], f"{float(r['AverageNs'])/1e3:.1f} us")
PY
done
RTSDS_LIB=$PWD/rtsds_amd/var_up4.so timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -k "upce or upsample_cross or ce_" >> $o 2>&1 || true
echo ok
