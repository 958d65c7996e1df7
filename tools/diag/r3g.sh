#!/bin/bash
# HIP runtime graph-launch settings vs. the multi-stream graph's host cost
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out
for env in "X=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" "DEBUG_HIP_GRAPH_BATCH_SIZE=8" "DEBUG_HIP_GRAPH_BATCH_SIZE=64" "DEBUG_HIP_GRAPH_BATCH_SIZE=512" "DEBUG_HIP_FORCE_GRAPH_QUEUES=2"; do
  echo "== $env" >> $o/r3g_env.txt
  env $env timeout -k 10 200 python -u tools/diag/enqueue.py --modes branches --steps 30 >> $o/r3g_env.txt 2>&1
done
echo ok
