#!/bin/bash
# narrow 1x1 data gradient tiling variants: parity, then the event-timed micro-bench per variant
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "pw" > gpurun_out/r6o_ops.txt 2>&1 || { tail -30 gpurun_out/r6o_ops.txt; exit 1; }
tail -1 gpurun_out/r6o_ops.txt
for v in base pw64 pwr4 pw8 base; do
  lib=$PWD/rtsds_amd/var_$v.so; [ "$v" = base ] && lib=$PWD/rtsds_amd/librtsds_hip.so
  RTSDS_LIB=$lib timeout -k 10 120 python3 tools/bench_pw.py || exit 1
done
