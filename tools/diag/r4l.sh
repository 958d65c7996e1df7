#!/bin/bash
# copy origins (train / inference) + full GPU suite
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 tools/diag/copy_origins.py bisenet-seg > gpurun_out/r4l_copies.txt 2>&1
timeout -k 10 300 python3 tools/diag/copy_origins.py bisenet-seg 8 infer >> gpurun_out/r4l_copies.txt 2>&1
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4l_pytest.log 2>&1
echo ok
