#!/bin/bash
# One-pass vector bilinear backward: parity (bit-identical to the two-pass kernels, torch fp64),
# model tests, whole-step A/B vs HEAD's ew unit and the kernel trace of both.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_ops_gpu.py -k "bilinear or concat or upsoftmax or resize" \
  tests/test_models_gpu.py > gpurun_out/r5ab_pytest.log 2>&1 || { tail -30 gpurun_out/r5ab_pytest.log; exit 1; }
tail -1 gpurun_out/r5ab_pytest.log
for v in base head base head base head; do
  lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
  RTSDS_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-conv-profile --no-infer > gpurun_out/r5ab_bench_$v.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r5ab_bench_$v.json $v | tee -a gpurun_out/r5ab_ab.txt
done
for v in base head; do
  lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
  RTSDS_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r5ab_$v -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-infer --no-conv-profile --submit branches > gpurun_out/r5ab_prof_$v.log 2>&1 || exit 1
  python3 tools/kstats.py $(ls /tmp/r5ab_$v/run_kernel_stats.csv) 6 > gpurun_out/r5ab_kstats_$v.txt
done
