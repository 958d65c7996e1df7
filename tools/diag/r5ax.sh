#!/bin/bash
# narrow pointwise weight gradient v2 (tools/variants/pww_prefetch.patch: x values prefetched into
# registers, 16-32 rows per workgroup) as rtsds_amd/var_head.so vs the in-tree split-K GEMM (base):
# parity of the variant (conv op cases, bench conv geometries), train conv report, bench A/B.
cd "$GRAFT_REPO_ROOT"
RTSDS_LIB=$PWD/rtsds_amd/var_head.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_ops_gpu.py::test_conv_fwd_bwd tests/test_configs_gpu.py::test_bench_conv_shapes > gpurun_out/r5ax_pytest.log 2>&1 || { tail -30 gpurun_out/r5ax_pytest.log; exit 1; }
tail -1 gpurun_out/r5ax_pytest.log
for v in base head; do
  lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
  RTSDS_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --conv-report --no-cpu-baseline --no-infer --steps 3 --warmup 2 > gpurun_out/r5ax_report_$v.txt 2>&1 || exit 1
  grep -E "wgrad .*x19 k1" gpurun_out/r5ax_report_$v.txt | sed "s/^/$v /"
done
for v in base head base head base head; do
  lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
  RTSDS_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-conv-profile --no-infer > gpurun_out/r5ax_bench_$v.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r5ax_bench_$v.json $v | tee -a gpurun_out/r5ax_ab.txt
done
