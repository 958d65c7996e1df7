#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/diag/infer_bf16.py 2 > gpurun_out/r4b_infer_bf16.txt 2>&1
timeout -k 10 300 python -u tools/diag/infer_bf16.py 8 >> gpurun_out/r4b_infer_bf16.txt 2>&1
echo ok
