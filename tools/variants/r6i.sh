#!/bin/bash
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ops_gpu.py -k "maxpool or stem or relu_maxpool" \
  tests/test_models_gpu.py -k "maxpool or stem or relu_maxpool or fp32_matches_oracle_and or seg_step_matches or graphed_step_equals_eager" > gpurun_out/r6i_pytest.log 2>&1 || { tail -30 gpurun_out/r6i_pytest.log; exit 1; }
tail -2 gpurun_out/r6i_pytest.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r6i_kt -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-infer --no-conv-profile > gpurun_out/r6i_bench_kt.log 2>&1
python3 tools/kstats.py $(ls /tmp/r6i_kt/run_kernel_stats.csv) 6 > gpurun_out/r6i_kernel_stats.txt
timeout -k 10 600 bash tools/ab_step.sh 2 base > gpurun_out/r6i_step.txt 2>&1
