#!/bin/bash
# sanity of the final in-tree library: smoke + conv / model op tests
set -e
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5zg_smoke.txt 2>&1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ops_gpu.py tests/test_models_gpu.py > gpurun_out/r5zg_pytest.log 2>&1
tail -1 gpurun_out/r5zg_smoke.txt; tail -1 gpurun_out/r5zg_pytest.log
