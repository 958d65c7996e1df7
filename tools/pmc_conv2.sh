#!/bin/bash
# Counter passes over one conv layer's fwd/dgrad/wgrad: pmc_conv2.sh TAG N C H W K KH S P
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=$1; shift
o=gpurun_out/pmc2_$tag; mkdir -p $o
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --output-format csv -d $o/sq -o run -- python3 tools/bench_conv.py "$@" 3 > $o/log 2>&1
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $o/tcc -o run -- python3 tools/bench_conv.py "$@" 3 >> $o/log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM --output-format csv -d $o/sq2 -o run -- python3 tools/bench_conv.py "$@" 3 >> $o/log 2>&1
