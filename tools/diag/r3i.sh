#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/r3i_pytest.log 2>&1
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $o/r3i_bench.json 2> $o/r3i_bench.err
echo ok
