#!/bin/bash
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 bash tools/ab_step.sh 3 base oldpool > gpurun_out/r6j_step.txt 2>&1
