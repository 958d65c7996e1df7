#!/bin/bash
# Round 5 session b: pipelined one-barrier conv loop + look-ahead fragment reads in the halo /
# image convs -- parity first, then conv-suite and whole-step (train + inference) A/B against
# the HEAD conv / hconv / imgconv units (rtsds_amd/var_head.so, tools/build_unit_rev.sh).
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  "tests/test_ops_gpu.py::test_conv_fwd_bwd" \
  "tests/test_configs_gpu.py::test_bisenet_bench_inference_bf16_blockwise" > gpurun_out/r5b_pytest.log 2>&1 || { tail -30 gpurun_out/r5b_pytest.log; exit 1; }
tail -3 gpurun_out/r5b_pytest.log
grep -A30 "teacher-forced stage errors" gpurun_out/r5b_pytest.log | head -30
for v in librtsds_hip var_head; do
  echo "== $v" >> gpurun_out/r5b_suite.txt
  timeout -k 10 300 bash tools/conv_suite.sh $PWD/rtsds_amd/$v.so >> gpurun_out/r5b_suite.txt 2>/dev/null || exit 1
done
for v in base head base head; do
  lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
  RTSDS_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-conv-profile > gpurun_out/r5b_bench_$v.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(sys.argv[2], d['value'], d['ms_per_step'], d.get('inference_fps_bs8'), d.get('inference_fps_bs1'))" gpurun_out/r5b_bench_$v.json $v | tee -a gpurun_out/r5b_ab.txt
done
