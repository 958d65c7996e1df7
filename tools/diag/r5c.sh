#!/bin/bash
# Kernel-trace A/B of the new conv / hconv / imgconv units vs HEAD (var_head.so): train step
# (bench.py, 10 steps) and the bs-8 inference forward (tools/diag/infer.py, 20 replays).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in base head; do
  lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
  r=/tmp/prof_r5c_$v; mkdir -p $r
  RTSDS_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $r/train -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-infer --no-conv-profile > gpurun_out/r5c_train_$v.log 2>&1 || exit 1
  python3 tools/kstats.py $r/train/run_kernel_stats.csv 14 --all > gpurun_out/r5c_train_$v.txt
  RTSDS_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $r/infer -o run -- python3 tools/diag/infer.py --reps 20 > gpurun_out/r5c_infer_$v.log 2>&1 || exit 1
  python3 tools/kstats.py $r/infer/run_kernel_stats.csv 25 --all > gpurun_out/r5c_infer_$v.txt
done
echo done
