#!/bin/bash
# rocprofv3 kernel-trace + stats of the bench (no CPU baseline), outputs under gpurun_out/prof_$1
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$1 -o run -- python3 bench.py --steps ${2:-5} --warmup 2 --no-cpu-baseline --no-infer > gpurun_out/prof_$1.log 2>&1
