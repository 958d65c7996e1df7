#!/bin/bash
# Two-K-team 128x128 WGRAD workgroups (half the split slabs): parity + determinism on every bench
# conv geometry, model tests, then whole-step A/B vs HEAD's conv units and split-reduce traffic.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_configs_gpu.py::test_bench_conv_shapes \
  tests/test_ops_gpu.py tests/test_models_gpu.py > gpurun_out/r5r_pytest.log 2>&1 || { tail -30 gpurun_out/r5r_pytest.log; exit 1; }
tail -1 gpurun_out/r5r_pytest.log
for v in base head base head base head; do
  lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
  RTSDS_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-conv-profile --no-infer > gpurun_out/r5r_bench_$v.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r5r_bench_$v.json $v | tee -a gpurun_out/r5r_ab.txt
done
for v in base head; do
  lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
  args="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-infer --no-conv-profile --submit branches"
  RTSDS_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r5r_$v/kt -o run -- python3 $args > gpurun_out/r5r_prof_$v.log 2>&1 || exit 1
  RTSDS_LIB=$PWD/$lib timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/r5r_$v/fetch -o run -- python3 $args >> gpurun_out/r5r_prof_$v.log 2>&1 || exit 1
  RTSDS_LIB=$PWD/$lib timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/r5r_$v/write -o run -- python3 $args >> gpurun_out/r5r_prof_$v.log 2>&1 || exit 1
  python3 tools/kstats.py $(ls /tmp/r5r_$v/kt/run_kernel_stats.csv) 6 > gpurun_out/r5r_kstats_$v.txt
  python3 tools/pmc_traffic.py /tmp/r5r_$v 6 > gpurun_out/r5r_traffic_$v.txt
done
