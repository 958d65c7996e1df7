#!/bin/bash
cd "$GRAFT_REPO_ROOT"


timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_models_gpu.py \
  -k "bf16_close or seg_step_matches or da_iterations or da2_epochs or fp32_matches_oracle_and" > gpurun_out/r6d_models.log 2>&1
