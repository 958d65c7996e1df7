#!/bin/bash
# Two taps per K-tile in the buffer-DMA forward (32-channel pitch: the discriminator's first conv)
# vs HEAD: parity on every bench geometry + conv ops + models, the conv shapes, DA bench A/B.
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_configs_gpu.py::test_bench_conv_shapes \
  tests/test_ops_gpu.py tests/test_models_gpu.py > gpurun_out/r5an_pytest.log 2>&1 || { tail -30 gpurun_out/r5an_pytest.log; exit 1; }
tail -1 gpurun_out/r5an_pytest.log
o=gpurun_out/r5an_conv.txt; : > $o
for a in "8 19 512 1024 64 4 2 1 10" "8 19 64 128 19 1 1 0 30"; do
  for v in base head; do
    lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
    echo "== $v" >> $o
    RTSDS_LIB=$PWD/$lib timeout -k 5 120 python3 tools/bench_conv.py $a 2>&1 | grep -E "fwd" >> $o || exit 1
  done
done
for v in base head base head; do
  lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
  RTSDS_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --workload bisenet-da --no-cpu-baseline --no-conv-profile --no-infer > gpurun_out/r5an_bench_$v.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r5an_bench_$v.json $v | tee -a gpurun_out/r5an_ab.txt
done
