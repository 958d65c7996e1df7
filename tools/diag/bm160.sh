set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_configs_gpu.py tests/test_ops_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "conv" > gpurun_out/bm160_pytest.log 2>&1
echo tests ok
bash tools/conv_suite.sh > gpurun_out/bm160_suite.log 2>&1
timeout -k 10 300 python3 bench.py --workload deeplab-seg --no-cpu-baseline > gpurun_out/bm160_dl.json 2>/dev/null
timeout -k 10 300 python3 bench.py --workload deeplab-da --no-cpu-baseline > gpurun_out/bm160_dlda.json 2>/dev/null
echo ok
