#!/bin/bash
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ops_gpu.py -k "into_slice or eval_fold or concat_resized or conv_fwd_bwd" \
  tests/test_models_gpu.py::test_bisenet_inference_fast_path_matches_general_path tests/test_configs_gpu.py -k "into_slice or eval_fold or concat_resized or conv_fwd_bwd or inference or eval_fast" > gpurun_out/r6e_pytest.log 2>&1 || { tail -30 gpurun_out/r6e_pytest.log; exit 1; }
tail -2 gpurun_out/r6e_pytest.log
timeout -k 10 300 python3 tools/ab_infer.py spatial_into_concat False True --rounds 4 > gpurun_out/r6e_infer.txt 2>&1
