#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/profile_all.sh r4t bisenet-seg
bash tools/profile_infer.sh r4t
echo ok
