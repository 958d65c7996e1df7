#!/bin/bash
# 8-wave 256 x 128 FWD tiles (3-deep ring): parity, then conv suite / per-conv report / bench
# A/B against the committed conv_gemm_fwd (rtsds_amd/var_head.so).
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_ops_gpu.py \
  "tests/test_configs_gpu.py::test_bench_conv_shapes" "tests/test_configs_gpu.py::test_bisenet_1024x512_fp32_forward_matches_oracle" \
  tests/test_models_gpu.py > gpurun_out/r5f_pytest.log 2>&1 || { tail -30 gpurun_out/r5f_pytest.log; exit 1; }
tail -2 gpurun_out/r5f_pytest.log
for v in librtsds_hip var_head; do
  echo "== $v" >> gpurun_out/r5f_suite.txt
  timeout -k 10 300 bash tools/conv_suite.sh $PWD/rtsds_amd/$v.so 2>/dev/null | grep fwd >> gpurun_out/r5f_suite.txt || exit 1
done
for v in base head base head; do
  lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
  RTSDS_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-conv-profile > gpurun_out/r5f_bench_$v.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(sys.argv[2], d['value'], d['ms_per_step'], d.get('inference_fps_bs8'), d.get('inference_fps_bs1'))" gpurun_out/r5f_bench_$v.json $v | tee -a gpurun_out/r5f_ab.txt
done
