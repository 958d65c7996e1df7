#!/bin/bash
# MFMA-utilisation counters of the bench's kernels (one rocprofv3 --pmc pass, SQ + GRBM blocks):
# SQ_VALU_MFMA_BUSY_CYCLES (cycles, summed over SIMDs), GRBM_GUI_ACTIVE (GPU-busy cycles, summed
# over the 8 XCDs), wave cycles / waits.  -> gpurun_out/pmc_mfma_$1/
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=${1:-r2}; shift || true
args="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-infer --no-conv-profile $*"
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_mfma_$tag -o run -- python3 $args > gpurun_out/pmc_mfma_$tag.log 2>&1
