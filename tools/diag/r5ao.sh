#!/bin/bash
# per-conv report at HEAD (train step + eval), for picking the next conv target
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --conv-report --no-cpu-baseline --steps 3 --warmup 2 > gpurun_out/r5ao_report.txt 2>&1
