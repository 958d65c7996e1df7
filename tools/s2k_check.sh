set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "conv or deeplab or dgrad or bottleneck" > gpurun_out/s2k_pytest.log 2>&1
bash tools/conv_suite.sh > gpurun_out/s2k_conv_suite.txt 2>&1
timeout -k 10 400 python -u bench.py --workload deeplab-seg --no-cpu-baseline --no-infer > gpurun_out/s2k_dl_bench.json 2> gpurun_out/s2k_dl_bench.err
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/s2k_bench.json 2> gpurun_out/s2k_bench.err
echo done
