#!/bin/bash
# 8-wave 256 x 128 FWD tiles (3-deep ring): parity, then conv suite / per-conv report / bench
# A/B against the committed conv_gemm_fwd (rtsds_amd/var_head.so).
cd "$GRAFT_REPO_ROOT"
for v in librtsds_hip var_head; do
  echo "== $v" >> gpurun_out/r5g_suite.txt
  timeout -k 10 300 bash tools/conv_suite.sh $PWD/rtsds_amd/$v.so 2>/dev/null | grep fwd >> gpurun_out/r5g_suite.txt || exit 1
done
for v in base head base head; do
  lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
  RTSDS_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-conv-profile > gpurun_out/r5g_bench_$v.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(sys.argv[2], d['value'], d['ms_per_step'], d.get('inference_fps_bs8'), d.get('inference_fps_bs1'))" gpurun_out/r5g_bench_$v.json $v | tee -a gpurun_out/r5g_ab.txt
done
for v in base head base head; do
  lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
  RTSDS_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --conv-report --no-cpu-baseline --steps 3 --warmup 2 > gpurun_out/r5g_report_${v}_$(date +%s%N).txt 2>&1 || exit 1
done
for w in deeplab-da bisenet-da deeplab-seg; do
  timeout -k 10 400 python3 bench.py --workload $w --no-cpu-baseline --no-conv-profile > gpurun_out/r5g_line_$w.json 2>gpurun_out/r5g_line_$w.err || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(sys.argv[2], d['value'], d['ms_per_step'], d.get('graph_submit'), d.get('graph_submit_trials'), d.get('host_launch_ms_per_step'))" gpurun_out/r5g_line_$w.json $w | tee -a gpurun_out/r5g_ab.txt
done
