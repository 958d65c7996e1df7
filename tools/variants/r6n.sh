#!/bin/bash
# pw_dgrad 4 rows per pass (accumulate operands prefetched): parity, kernel times, step vs previous Python
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "pw or conv_cases or bench_conv" > gpurun_out/r6n_ops.txt 2>&1 || { tail -30 gpurun_out/r6n_ops.txt; exit 1; }
tail -2 gpurun_out/r6n_ops.txt
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_models_gpu.py -k "supervision_joins or seg_step" > gpurun_out/r6n_tests.txt 2>&1 || { tail -30 gpurun_out/r6n_tests.txt; exit 1; }
tail -2 gpurun_out/r6n_tests.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6n_prof -o run -- python3 bench.py --no-cpu-baseline --no-conv-profile --no-infer --steps 10 --warmup 3 > gpurun_out/r6n_bench.json 2>/dev/null || exit 1
timeout -k 10 1200 bash tools/ab_tree.sh 4 > gpurun_out/r6n_step.txt 2>&1; cat gpurun_out/r6n_step.txt
