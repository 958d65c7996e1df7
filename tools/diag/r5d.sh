#!/bin/bash
# Per-conv event-timed table of the train step and the eval forward (bench.py --conv-report),
# new units vs HEAD (var_head.so), twice each.
cd "$GRAFT_REPO_ROOT"
for v in base head base head; do
  lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
  RTSDS_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --conv-report --no-cpu-baseline --steps 3 --warmup 2 > gpurun_out/r5d_report_$v.txt 2>&1 || exit 1
  cp gpurun_out/r5d_report_$v.txt gpurun_out/r5d_report_${v}_$(date +%s).txt
done
echo done
