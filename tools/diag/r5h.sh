#!/bin/bash
# Two-barrier schedule with look-ahead fragment reads for the non-ring tiles (base) vs the
# compiler-scheduled reads (var_old2, -DCDIAG_OLD2): parity, per-conv report and bench A/B.
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "tests/test_ops_gpu.py" \
  "tests/test_configs_gpu.py::test_bench_conv_shapes" > gpurun_out/r5h_pytest.log 2>&1 || { tail -30 gpurun_out/r5h_pytest.log; exit 1; }
tail -1 gpurun_out/r5h_pytest.log
for v in base old2 base old2; do
  lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
  RTSDS_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --conv-report --no-cpu-baseline --steps 3 --warmup 2 > gpurun_out/r5h_report_${v}_$(date +%s%N).txt 2>&1 || exit 1
done
for v in base old2 base old2; do
  lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
  RTSDS_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-conv-profile > gpurun_out/r5h_bench_$v.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(sys.argv[2], d['value'], d['ms_per_step'], d.get('inference_fps_bs8'), d.get('inference_fps_bs1'))" gpurun_out/r5h_bench_$v.json $v | tee -a gpurun_out/r5h_ab.txt
done
