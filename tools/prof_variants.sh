#!/bin/bash
# kernel-trace the bench once per library variant: prof_variants.sh TAG base v1 v2 ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=$1; shift
for v in "$@"; do
  lib=$PWD/rtsds_amd/var_$v.so; [ "$v" = base ] && lib=$PWD/rtsds_amd/librtsds_hip.so
  RTSDS_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pv_${tag}_$v -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-infer > gpurun_out/pv_${tag}_$v.log 2>&1 || exit 1
done
