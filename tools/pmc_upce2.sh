#!/bin/bash
# kernel trace + SQ/LDS counters of the fused upsample+CE micro-benchmark -> gpurun_out/pmc_upce2_$1
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/pmc_upce2_$1; mkdir -p $o
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $o/kt -o run -- python3 tools/bench_upce.py 10 > $o/log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES --output-format csv -d $o/sq -o run -- python3 tools/bench_upce.py 4 >> $o/log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_TRANS_F32 GRBM_GUI_ACTIVE --output-format csv -d $o/sq2 -o run -- python3 tools/bench_upce.py 4 >> $o/log 2>&1
