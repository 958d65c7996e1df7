#!/bin/bash
# kernel-trace summary of one conv layer's fwd/dgrad/wgrad: kt_conv.sh TAG N C H W K KH S P
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=$1; shift
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_conv_$tag -o run -- python3 tools/bench_conv.py "$@" 20 > gpurun_out/kt_conv_$tag.log 2>&1
