#!/bin/bash
# round-6 final evidence, part 2 (refreshed at the final HEAD): per-workload kernel / traffic / MFMA profiles + inference
cd "$GRAFT_REPO_ROOT"
timeout -k 10 1000 bash tools/profile_all.sh r6zj && timeout -k 10 400 bash tools/profile_infer.sh r6zj
