#!/bin/bash
# feature joins (layer-3 output, tail) + pooled dgrad accumulate rounding: parity, then the step vs the previous revision's Python
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "batchnorm or concat or bn_ or pooled or chscale or gap" > gpurun_out/r6s_ops.txt 2>&1 || { tail -30 gpurun_out/r6s_ops.txt; exit 1; }
tail -1 gpurun_out/r6s_ops.txt
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_models_gpu.py -k "bisenet or seg_step or graphed_step_equals_eager or da_iterations or da_step or side_stream" > gpurun_out/r6s_models.txt 2>&1 || { tail -30 gpurun_out/r6s_models.txt; exit 1; }
tail -1 gpurun_out/r6s_models.txt
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_configs_gpu.py -k "bisenet" > gpurun_out/r6s_configs.txt 2>&1 || { tail -30 gpurun_out/r6s_configs.txt; exit 1; }
tail -1 gpurun_out/r6s_configs.txt
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_dp_gpu.py > gpurun_out/r6s_dp.txt 2>&1 || { tail -30 gpurun_out/r6s_dp.txt; exit 1; }
tail -1 gpurun_out/r6s_dp.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6s_prof -o run -- python3 bench.py --no-cpu-baseline --no-conv-profile --no-infer --steps 10 --warmup 3 > gpurun_out/r6s_bench.json 2>/dev/null || exit 1
timeout -k 10 1200 bash tools/ab_tree.sh 4 > gpurun_out/r6s_step.txt 2>&1; cat gpurun_out/r6s_step.txt
