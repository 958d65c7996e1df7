#!/bin/bash
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 tools/ab_infer.py eval_branch_batch 0 4 --rounds 4 > gpurun_out/r6d_infer.txt 2>&1
