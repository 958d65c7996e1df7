#!/bin/bash
# GPU check of a conv-kernel change: the conv op / bench-geometry parity tests, then the conv
# micro-benchmarks of the working tree (base) against saved libraries: r6_conv_check.sh TAG [variants]
cd "$GRAFT_REPO_ROOT"
tag=$1; shift
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ops_gpu.py -k "conv" \
  tests/test_configs_gpu.py::test_bench_conv_shapes > gpurun_out/${tag}_pytest.log 2>&1 || { tail -30 gpurun_out/${tag}_pytest.log; exit 1; }
tail -3 gpurun_out/${tag}_pytest.log
timeout -k 10 600 bash tools/variants/run_conv_diag.sh "$@" > gpurun_out/${tag}_conv.txt 2>&1
