#!/bin/bash
# supervision GradJoins + overwritten accuracy count + cached backward seed: parity, then the
# whole step against the previous revision's Python on the same library (tools/ab_tree.sh)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_models_gpu.py -k "supervision_joins or seg_step or graphed_step_equals_eager or branch_streams or bisenet_fp32 or da_iterations" > gpurun_out/r6l_tests.txt 2>&1 || { tail -30 gpurun_out/r6l_tests.txt; exit 1; }
tail -2 gpurun_out/r6l_tests.txt
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "upce or pw or conv_pointwise or bilinear or cat" > gpurun_out/r6l_ops.txt 2>&1 || { tail -30 gpurun_out/r6l_ops.txt; exit 1; }
tail -2 gpurun_out/r6l_ops.txt
timeout -k 10 900 bash tools/ab_tree.sh 3 > gpurun_out/r6l_step.txt 2>&1; cat gpurun_out/r6l_step.txt
