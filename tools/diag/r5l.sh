#!/bin/bash
# tapwgrad v2 (one barrier per tile, DMA pieces between MFMA groups, 16-B slab stores) vs a03ae5f
# against HEAD's conv / tapconv units (rtsds_amd/var_head.so).
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "tests/test_ops_gpu.py::test_tapconv_partial_tiles" \
  tests/test_models_gpu.py > gpurun_out/r5l_pytest.log 2>&1 || { tail -30 gpurun_out/r5l_pytest.log; exit 1; }
tail -1 gpurun_out/r5l_pytest.log
for v in base head base head; do
  lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
  RTSDS_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --conv-report --no-cpu-baseline --no-infer --steps 3 --warmup 2 > gpurun_out/r5l_report_${v}_$(date +%s%N).txt 2>&1 || exit 1
done
for v in base head base head; do
  lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
  RTSDS_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-conv-profile --no-infer > gpurun_out/r5l_bench_$v.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r5l_bench_$v.json $v | tee -a gpurun_out/r5l_ab.txt
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in base head; do
  lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
  RTSDS_LIB=$PWD/$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r5l_$v -o run -- python3 tools/bench_conv.py 8 64 128 256 64 3 1 1 30 > gpurun_out/r5l_k_$v.log 2>&1 || exit 1
  python3 tools/kstats.py /tmp/r5l_$v/run_kernel_stats.csv 33 > gpurun_out/r5l_k_$v.txt
done
