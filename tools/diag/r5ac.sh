#!/bin/bash
# kernel trace of the bench step (graph replay) for the step timeline (tools/diag/step_timeline.py)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/r5ac -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-infer --no-conv-profile --submit branches > gpurun_out/r5ac.log 2>&1 || exit 1
cp $(ls /tmp/r5ac/run_kernel_trace.csv) gpurun_out/r5ac_kernel_trace.csv
python3 tools/diag/step_timeline.py gpurun_out/r5ac_kernel_trace.csv 25 > gpurun_out/r5ac_timeline.txt
