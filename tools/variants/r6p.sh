#!/bin/bash
# BatchNorm backward statistics row blocks (512 -> 1024, U 2 -> 4): kernel totals per variant, then the whole step
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "bn" > gpurun_out/r6p_ops.txt 2>&1 || { tail -30 gpurun_out/r6p_ops.txt; exit 1; }
tail -1 gpurun_out/r6p_ops.txt
for v in base bnrb1k bnrb1ku4; do
  lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
  RTSDS_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6p_prof_$v -o run -- python3 bench.py --no-cpu-baseline --no-conv-profile --no-infer --steps 10 --warmup 3 > gpurun_out/r6p_bench_$v.json 2>/dev/null || exit 1
done
timeout -k 10 1200 bash tools/ab_step.sh 3 base bnrb1k bnrb1ku4 > gpurun_out/r6p_step.txt 2>&1; cat gpurun_out/r6p_step.txt
