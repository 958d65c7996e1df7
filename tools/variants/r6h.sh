#!/bin/bash
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ops_gpu.py tests/test_models_gpu.py tests/test_configs_gpu.py \
  -k "ffm_head or into_slice or eval_fold or concat_resized or inference or eval_fast" > gpurun_out/r6h_pytest.log 2>&1 || { tail -30 gpurun_out/r6h_pytest.log; exit 1; }
tail -2 gpurun_out/r6h_pytest.log
timeout -k 10 600 bash tools/profile_infer.sh r6h > gpurun_out/r6h_prof.log 2>&1
