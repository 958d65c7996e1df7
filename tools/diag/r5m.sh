#!/bin/bash
# PMC passes of the layer1 direct weight-gradient kernel (tapwgrad_kernel): where its cycles go
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r5m; mkdir -p $o
a="tools/bench_conv.py 8 64 128 256 64 3 1 1 10"
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d /tmp/r5m/p1 -o run -- python3 $a > $o/log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d /tmp/r5m/p2 -o run -- python3 $a >> $o/log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum --output-format csv -d /tmp/r5m/p3 -o run -- python3 $a >> $o/log 2>&1 || exit 1
for p in p1 p2 p3; do python3 tools/pmc_summary.py $(ls /tmp/r5m/$p/run_counter_collection.csv) tapwgrad >> $o/summary.txt; python3 tools/pmc_summary.py $(ls /tmp/r5m/$p/run_counter_collection.csv) split_reduce >> $o/summary.txt; done
