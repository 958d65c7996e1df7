#!/bin/bash
# upce kernel time per library variant: upce_variants.sh base v1 v2 ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  lib=$PWD/rtsds_amd/var_$v.so; [ "$v" = base ] && lib=$PWD/rtsds_amd/librtsds_hip.so
  RTSDS_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/uv_$v -o run -- python3 tools/bench_upce.py 20 > gpurun_out/uv_$v.log 2>&1 || exit 1
  echo "== $v"; grep -h upce gpurun_out/uv_$v/run_kernel_stats.csv | cut -d, -f1-5
done
