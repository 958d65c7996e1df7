#!/bin/bash
# One bench line per BASELINE.json workload (1 GPU) -> gpurun_out/wl_<tag>_<workload>.json
set -e
cd "$GRAFT_REPO_ROOT"
tag=${1:-r1}
for wl in bisenet-da deeplab-seg deeplab-da; do
  timeout -k 10 400 python -u bench.py --workload $wl --steps ${2:-10} --warmup 3 --no-cpu-baseline > gpurun_out/wl_${tag}_$wl.json 2> gpurun_out/wl_${tag}_$wl.err
done
echo done
