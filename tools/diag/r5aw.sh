#!/bin/bash
# narrow pointwise weight gradient (pww_kernel: the 19-class head 1x1 convs) vs the split-K GEMM (base):
# parity, train conv report, bench A/B.
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ops_gpu.py tests/test_models_gpu.py \
  tests/test_configs_gpu.py > gpurun_out/r5aw_pytest.log 2>&1 || { tail -30 gpurun_out/r5aw_pytest.log; exit 1; }
tail -1 gpurun_out/r5aw_pytest.log
for v in base head; do
  lib=rtsds_amd/var_$v.so; [ "$v" = head ] && lib=rtsds_amd/librtsds_hip.so
  RTSDS_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --conv-report --no-cpu-baseline --steps 3 --warmup 2 > gpurun_out/r5aw_report_$v.txt 2>&1 || exit 1
  grep -E "wgrad .*(x19|->.*x19) k1" gpurun_out/r5aw_report_$v.txt | sed "s/^/$v /"
done
for v in base head base head base head; do
  lib=rtsds_amd/var_$v.so; [ "$v" = head ] && lib=rtsds_amd/librtsds_hip.so
  RTSDS_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-conv-profile > gpurun_out/r5aw_bench_$v.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(sys.argv[2], d['value'], d['ms_per_step'], d['inference_fps_bs8'], d['inference_fps_bs1'])" gpurun_out/r5aw_bench_$v.json $v | tee -a gpurun_out/r5aw_ab.txt
done
