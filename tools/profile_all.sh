#!/bin/bash
# Round evidence for every bench workload: rocprofv3 kernel-trace stats, FETCH_SIZE and
# WRITE_SIZE passes (HBM traffic), and the MFMA-utilisation pass.  Outputs under
# gpurun_out/prof_<tag>_<workload>/ (summarise with tools/kstats.py, pmc_traffic.py,
# pmc_mfma_summary.py).  usage: profile_all.sh TAG [workload ...]
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=$1; shift
# heartbeat: PMC passes print nothing for minutes on the larger workloads
( while sleep 50; do date >> gpurun_out/prof_${tag}_heartbeat; done ) &
hb=$!
trap "kill $hb" EXIT
wls=${@:-bisenet-seg bisenet-da deeplab-seg deeplab-da}
for wl in $wls; do
  o=gpurun_out/prof_${tag}_$wl; mkdir -p $o
  args="bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline --no-infer --no-conv-profile"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/kt -o run -- python3 $args > $o/log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/fetch -o run -- python3 $args >> $o/log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/write -o run -- python3 $args >> $o/log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $o/mfma -o run -- python3 $args >> $o/log 2>&1
  echo "$wl done"
done
