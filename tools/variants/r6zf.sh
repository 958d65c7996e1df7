#!/bin/bash
# final evidence at HEAD: focused tests, full GPU suite, smoke, bench
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_ops_gpu.py tests/test_models_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "hconv or upsample_cross_entropy" > gpurun_out/r6zf_focus.txt 2>&1 || { tail -30 gpurun_out/r6zf_focus.txt; exit 1; }
tail -2 gpurun_out/r6zf_focus.txt
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6zf_gpu_tests.txt 2>&1 || { tail -30 gpurun_out/r6zf_gpu_tests.txt; exit 1; }
tail -3 gpurun_out/r6zf_gpu_tests.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6zf_smoke.txt 2>&1 || { tail -20 gpurun_out/r6zf_smoke.txt; exit 1; }
tail -3 gpurun_out/r6zf_smoke.txt
timeout -k 10 400 python3 bench.py > gpurun_out/r6zf_bench.json 2> gpurun_out/r6zf_bench.err || { tail -20 gpurun_out/r6zf_bench.err; exit 1; }
cat gpurun_out/r6zf_bench.json
