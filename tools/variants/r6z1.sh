#!/bin/bash
# round-6 final evidence, part 1: GPU suite, smoke, default bench line
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6z_gpu_tests.txt 2>&1 || { tail -30 gpurun_out/r6z_gpu_tests.txt; exit 1; }
tail -3 gpurun_out/r6z_gpu_tests.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6z_smoke.txt 2>&1 || { tail -20 gpurun_out/r6z_smoke.txt; exit 1; }
tail -3 gpurun_out/r6z_smoke.txt
timeout -k 10 400 python3 bench.py > gpurun_out/r6z_bench.json 2> gpurun_out/r6z_bench.err || { tail -20 gpurun_out/r6z_bench.err; exit 1; }
cat gpurun_out/r6z_bench.json
