#!/bin/bash
# split-K reductions batched 32 per launch (one launch per step) vs 16: op tests,
# bit identity against the previous conv.hip (tools/param_hash.py under both builds), kernel counts, step A/B
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_models_gpu.py -k "deferred_wgrad or side_stream_wgrad" > gpurun_out/r6zh_ops.txt 2>&1 || { tail -30 gpurun_out/r6zh_ops.txt; exit 1; }
tail -1 gpurun_out/r6zh_ops.txt
for v in base oldred; do
  lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
  RTSDS_LIB=$PWD/$lib timeout -k 10 300 python3 tools/param_hash.py > gpurun_out/r6zh_hash_$v.txt 2>&1 || { tail -20 gpurun_out/r6zh_hash_$v.txt; exit 1; }
done
cat gpurun_out/r6zh_hash_base.txt gpurun_out/r6zh_hash_oldred.txt | grep -v amdgpu.ids
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_models_gpu.py -k "bisenet or seg_step or graphed_step_equals_eager or da_iterations or deeplab" > gpurun_out/r6zh_models.txt 2>&1 || { tail -30 gpurun_out/r6zh_models.txt; exit 1; }
tail -1 gpurun_out/r6zh_models.txt
for v in base oldred; do
  lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
  RTSDS_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6zh_prof_$v -o run -- python3 bench.py --no-cpu-baseline --no-conv-profile --no-infer --steps 10 --warmup 3 > gpurun_out/r6zh_bench_$v.json 2>/dev/null || exit 1
done
timeout -k 10 900 bash tools/ab_step.sh 3 base oldred > gpurun_out/r6zh_step.txt 2>&1; cat gpurun_out/r6zh_step.txt
