#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 bench.py --steps 20 --no-cpu-baseline --conv-report > gpurun_out/r4aa_bench.json 2> gpurun_out/r4aa_conv_report.txt
echo ok
