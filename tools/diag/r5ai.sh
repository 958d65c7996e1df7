#!/bin/bash
# 256 x 64 DGRAD tiles for N = 64 data gradients with >= 2 rounds of them (spatial conv2) vs HEAD
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_configs_gpu.py::test_bench_conv_shapes \
  tests/test_ops_gpu.py -k "conv or bench_conv" > gpurun_out/r5ai_pytest.log 2>&1 || { tail -30 gpurun_out/r5ai_pytest.log; exit 1; }
tail -1 gpurun_out/r5ai_pytest.log
o=gpurun_out/r5ai_conv.txt; : > $o
for a in "8 64 256 512 128 3 2 1 30" "8 64 128 256 64 3 1 1 30"; do
  for v in base head; do
    lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
    echo "== $v" >> $o
    RTSDS_LIB=$PWD/$lib timeout -k 5 60 python3 tools/bench_conv.py $a 2>&1 | grep dgrad >> $o || exit 1
  done
done
for v in base head base head base head; do
  lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
  RTSDS_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-conv-profile --no-infer > gpurun_out/r5ai_bench_$v.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r5ai_bench_$v.json $v | tee -a gpurun_out/r5ai_ab.txt
done
