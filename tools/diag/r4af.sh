#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4af_pytest.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r4af_bench.json 2> gpurun_out/r4af_bench.err
timeout -k 10 300 python -u bench.py --workload bisenet-da --no-cpu-baseline --no-conv-profile > gpurun_out/r4af_bench_da.json 2> gpurun_out/r4af_bench_da.err
echo ok
