#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u bench.py --steps 20 --no-cpu-baseline --no-infer --conv-report > gpurun_out/r4d_bench.json 2> gpurun_out/r4d_conv_report.txt
timeout -k 10 300 python -u -m pytest tests/test_transforms_gpu.py -m gpu -q --timeout 120 --timeout-method thread -k "fixture" > gpurun_out/r4d_pytest.log 2>&1 || echo "pytest failed"
echo ok
