#!/bin/bash
# round 4: new parity tests (inference fast path vs oracle, bf16 inference vs fp32, fp16 wire
# all-reduce) + the default bench line with the inference roofline
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_configs_gpu.py tests/test_dp_gpu.py -m gpu -v -s --timeout 300 --timeout-method thread -k "eval_fast_path or inference_bf16 or fp16_wire or two_rank" > $o/r4a_pytest.log 2>&1 || echo "pytest failed"
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $o/r4a_bench.json 2> $o/r4a_bench.err
echo ok
