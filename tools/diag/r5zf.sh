#!/bin/bash
# round-5 final evidence at HEAD: GPU suite, smoke, default bench line, inference profile
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r5z_gpu_pytest.log 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5z_smoke.txt 2>&1
timeout -k 10 300 python3 -u bench.py > gpurun_out/r5z_bench_default.json 2> gpurun_out/r5z_bench_default.err
bash tools/profile_infer.sh r5z
echo ok
