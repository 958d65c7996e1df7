#!/bin/bash
# GPU test pass (+ optional test selection) -> gpurun_out/<tag>_pytest.log
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-t}; shift || true
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=25 "$@" > gpurun_out/${tag}_pytest.log 2>&1
echo done
