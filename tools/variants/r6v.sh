#!/bin/bash
# narrow pointwise weight + bias gradient route: parity, kernel times (base vs oldpwn), step A/B
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ops_gpu.py -k "conv or pw or bias" > gpurun_out/r6v_ops.txt 2>&1 || { tail -30 gpurun_out/r6v_ops.txt; exit 1; }
tail -1 gpurun_out/r6v_ops.txt
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_models_gpu.py -k "graphed_step_equals_eager or seg_step or bisenet_fp32 or feature_joins" > gpurun_out/r6v_models.txt 2>&1 || { tail -30 gpurun_out/r6v_models.txt; exit 1; }
tail -1 gpurun_out/r6v_models.txt
for v in base oldpwn; do
  lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
  RTSDS_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6v_prof_$v -o run -- python3 bench.py --no-cpu-baseline --no-conv-profile --no-infer --steps 10 --warmup 3 > gpurun_out/r6v_bench_$v.json 2>/dev/null || exit 1
done
timeout -k 10 900 bash tools/ab_step.sh 3 base oldpwn > gpurun_out/r6v_step.txt 2>&1; cat gpurun_out/r6v_step.txt
