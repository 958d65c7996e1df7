#!/bin/bash
# One bench line per workload -> gpurun_out/<tag>_bench_<workload>.json (+ .log)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=$1; shift
wls=${@:-bisenet-seg bisenet-da deeplab-seg deeplab-da}
for wl in $wls; do
  timeout -k 10 600 python3 -u bench.py --workload $wl > gpurun_out/${tag}_bench_$wl.json 2> gpurun_out/${tag}_bench_$wl.log
  cat gpurun_out/${tag}_bench_$wl.json
done
