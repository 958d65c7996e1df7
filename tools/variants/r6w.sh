#!/bin/bash
# FFM attention backward in one launch: parity, then the step against the previous revision (library and Python)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_models_gpu.py -k "fused_attention or bisenet_fp32 or seg_step or graphed_step_equals_eager or feature_joins or da_iterations" > gpurun_out/r6w_models.txt 2>&1 || { tail -30 gpurun_out/r6w_models.txt; exit 1; }
tail -1 gpurun_out/r6w_models.txt
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_configs_gpu.py -k "bisenet" tests/test_dp_gpu.py > gpurun_out/r6w_configs.txt 2>&1 || { tail -30 gpurun_out/r6w_configs.txt; exit 1; }
tail -1 gpurun_out/r6w_configs.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6w_prof -o run -- python3 bench.py --no-cpu-baseline --no-conv-profile --no-infer --steps 10 --warmup 3 > gpurun_out/r6w_bench.json 2>/dev/null || exit 1
timeout -k 10 1200 bash tools/ab_py_attr.sh 3 > gpurun_out/r6w_step.txt 2>&1; cat gpurun_out/r6w_step.txt
