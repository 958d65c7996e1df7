#!/bin/bash
# conv forward +stats cost: channel-major vs row-major (probe) partial stores
cd "$GRAFT_REPO_ROOT"
for r in 1 2; do for v in base rowm; do echo "== $v"; lib=$PWD/rtsds_amd/var_$v.so; [ $v = base ] && lib=$PWD/rtsds_amd/librtsds_hip.so; bash tools/conv_stats_suite.sh $lib; done; done
