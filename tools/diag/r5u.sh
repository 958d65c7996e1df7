#!/bin/bash
# upce_fwd counters (auxiliary-wave build): where the wave cycles go
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r5u; mkdir -p $o
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d /tmp/r5u/p1 -o run -- python3 tools/bench_upce.py 6 > $o/log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d /tmp/r5u/p2 -o run -- python3 tools/bench_upce.py 6 >> $o/log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_VMEM SQ_INSTS_SMEM --output-format csv -d /tmp/r5u/p3 -o run -- python3 tools/bench_upce.py 6 >> $o/log 2>&1 || exit 1
for p in p1 p2 p3; do python3 tools/pmc_summary.py $(ls /tmp/r5u/$p/run_counter_collection.csv) upce_fwd >> $o/summary.txt; done
