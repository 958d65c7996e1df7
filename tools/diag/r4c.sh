#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_configs_gpu.py -m gpu -v -s --timeout 300 --timeout-method thread -k "inference_bf16" > gpurun_out/r4c_pytest.log 2>&1 || echo "pytest failed"
echo ok
