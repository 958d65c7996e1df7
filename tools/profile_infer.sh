#!/bin/bash
# Inference-forward evidence: rocprofv3 kernel-trace stats and the MFMA /
# wait counter pass of the bs-8 eval forward replayed as a hipGraph (tools/diag/infer.py, 20
# replays + 3 warm-up + the capture's 2 eager warm-ups).  usage: profile_infer.sh TAG
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=$1
o=gpurun_out/prof_${tag}_infer; r=/tmp/prof_${tag}/infer; mkdir -p $o $r
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $r/kt -o run -- python3 tools/diag/infer.py --reps 20 > $o/log 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $r/mfma -o run -- python3 tools/diag/infer.py --reps 20 >> $o/log 2>&1
python3 tools/kstats.py $(ls $r/kt/run_kernel_stats.csv) 25 > $o/kernel_stats.txt
python3 tools/pmc_mfma_summary.py $(ls $r/mfma/run_counter_collection.csv) 25 > $o/mfma.txt
timeout -k 10 120 python3 tools/diag/infer.py --reps 50 > $o/fps.txt 2>&1
timeout -k 10 120 python3 tools/diag/infer.py --reps 200 --batch 1 >> $o/fps.txt 2>&1
echo "infer done"
