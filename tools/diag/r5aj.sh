#!/bin/bash
# upce row loop unrolled by 2 vs HEAD: parity, kernel times, bench A/B
# times (tools/bench_upce.py) and whole-step A/B vs HEAD's upce unit.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_ops_gpu.py -k "upsample_cross_entropy or upce" \
  tests/test_models_gpu.py tests/test_configs_gpu.py -k "upsample_cross_entropy or upce or bisenet or seg_iteration or da_iteration" > gpurun_out/r5aj_pytest.log 2>&1 || { tail -30 gpurun_out/r5aj_pytest.log; exit 1; }
tail -1 gpurun_out/r5aj_pytest.log
for v in base head base head; do
  lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
  RTSDS_LIB=$PWD/$lib timeout -k 10 120 python3 tools/bench_upce.py 20 >> gpurun_out/r5aj_upce_$v.txt 2>&1 || exit 1
done
for v in base head base head base head; do
  lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
  RTSDS_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-conv-profile --no-infer > gpurun_out/r5aj_bench_$v.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r5aj_bench_$v.json $v | tee -a gpurun_out/r5aj_ab.txt
done
for v in base head; do
  lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
  RTSDS_LIB=$PWD/$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r5aj_$v -o run -- python3 tools/bench_upce.py 20 > gpurun_out/r5aj_k_$v.log 2>&1 || exit 1
  python3 tools/kstats.py $(ls /tmp/r5aj_$v/run_kernel_stats.csv) 20 > gpurun_out/r5aj_k_$v.txt
done
