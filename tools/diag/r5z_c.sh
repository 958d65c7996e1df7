#!/bin/bash
# round-5 (end of session) evidence, part C: DeepLab profiles
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/profile_all.sh r5z deeplab-seg deeplab-da
echo ok
