#!/bin/bash
# counters of the tapconv forward vs the GEMM forward at the BiSeNet layer1 geometry
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r4f; mkdir -p $o
for lib in librtsds_hip var_notap; do
  export RTSDS_LIB=$PWD/rtsds_amd/$lib.so
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r4f/$lib/kt -o run -- python3 tools/diag/conv_one.py fwd 8 64 128 256 64 3 1 1 20 > $o/${lib}_kt.log 2>&1
  timeout -s KILL 60 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d /tmp/r4f/$lib/pmc -o run -- python3 tools/diag/conv_one.py fwd 8 64 128 256 64 3 1 1 20 > $o/${lib}_pmc.log 2>&1
  timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d /tmp/r4f/$lib/pmc2 -o run -- python3 tools/diag/conv_one.py fwd 8 64 128 256 64 3 1 1 20 > $o/${lib}_pmc2.log 2>&1
  cp /tmp/r4f/$lib/kt/run_kernel_stats.csv $o/${lib}_kernel_stats.csv
  cp /tmp/r4f/$lib/pmc/run_counter_collection.csv $o/${lib}_pmc.csv
  cp /tmp/r4f/$lib/pmc2/run_counter_collection.csv $o/${lib}_pmc2.csv
done
echo ok
