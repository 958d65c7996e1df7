#!/bin/bash
# rocprofv3 kernel trace + SQ counters of one conv layer: pmc_conv.sh TAG N C H W K KH S P
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=$1; shift
timeout -k 10 300 python3 tools/bench_conv.py "$@" 20 > gpurun_out/pmc_conv_$tag.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --output-format csv -d gpurun_out/pmc_conv_$tag/pmc -o run -- python3 tools/bench_conv.py "$@" 3 >> gpurun_out/pmc_conv_$tag.log 2>&1
