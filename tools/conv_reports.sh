#!/bin/bash
# Per-layer conv tables for the BiSeNet and DeepLab seg workloads + the conv micro-suite
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=$1
for wl in bisenet-seg deeplab-seg; do
  timeout -k 10 400 python -u bench.py --workload $wl --steps 2 --warmup 1 --no-cpu-baseline --no-infer --conv-report > gpurun_out/${tag}_${wl}_report.json 2> gpurun_out/${tag}_${wl}_report.txt
  python3 tools/conv_table.py gpurun_out/${tag}_${wl}_report.txt 25 > gpurun_out/${tag}_${wl}_conv_layers.md
done
bash tools/conv_suite.sh > gpurun_out/${tag}_conv_suite.txt 2>&1
echo done
