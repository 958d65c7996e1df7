#!/bin/bash
# Per-tile loop choice (pipelined one-barrier loop for FWD / WGRAD >= 128 x 128 only), hconv
# two-tap look-ahead, imgconv_pool reverted: parity, then per-conv report + bench A/B vs HEAD.
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r5e_pytest.log 2>&1 || { tail -30 gpurun_out/r5e_pytest.log; exit 1; }
tail -2 gpurun_out/r5e_pytest.log
for v in base head base head; do
  lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
  RTSDS_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --conv-report --no-cpu-baseline --steps 3 --warmup 2 > gpurun_out/r5e_report_${v}_$(date +%s%N).txt 2>&1 || exit 1
done
for v in base head base head; do
  lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
  RTSDS_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-conv-profile > gpurun_out/r5e_bench_$v.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(sys.argv[2], d['value'], d['ms_per_step'], d.get('inference_fps_bs8'), d.get('inference_fps_bs1'))" gpurun_out/r5e_bench_$v.json $v | tee -a gpurun_out/r5e_ab.txt
done
# operand-bytes diagnostic (timing only, wrong results): FWD without the A / without the B DMA
for v in librtsds_hip var_noa var_nob; do
  echo "== $v" >> gpurun_out/r5e_bytes.txt
  timeout -k 10 300 bash tools/conv_suite.sh $PWD/rtsds_amd/$v.so 2>/dev/null | grep fwd >> gpurun_out/r5e_bytes.txt || exit 1
done
