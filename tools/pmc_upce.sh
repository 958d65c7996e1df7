#!/bin/bash
# SQ counter pass over the fused upsample+CE micro-benchmark -> gpurun_out/pmc_upce_$1
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc_upce_$1/kt -o run -- python3 tools/bench_upce.py 10 > gpurun_out/pmc_upce_$1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES --output-format csv -d gpurun_out/pmc_upce_$1/pmc -o run -- python3 tools/bench_upce.py 4 >> gpurun_out/pmc_upce_$1.log 2>&1
