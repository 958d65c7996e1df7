#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/pmc_upce2.sh r4al
o=gpurun_out/pmc_upce2_r4al
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES --output-format csv -d $o/sq3 -o run -- python3 tools/bench_upce.py 4 >> $o/log 2>&1 || echo "sq3 pass failed"
python3 tools/diag/upce_pmc_summary.py $o > $o/summary.txt
python3 tools/kstats.py $(ls $o/kt/run_kernel_stats.csv) 1 | head -5 >> $o/summary.txt
echo ok
