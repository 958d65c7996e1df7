#!/bin/bash
# Round evidence for every bench workload: rocprofv3 kernel-trace stats, FETCH_SIZE and
# WRITE_SIZE passes (HBM traffic), and the MFMA-utilisation pass.  Raw rocprofv3 output stays
# under /tmp on the box; the summaries (tools/kstats.py, pmc_traffic.py, pmc_mfma_summary.py)
# land in gpurun_out/prof_<tag>_<workload>/.  usage: profile_all.sh TAG [workload ...]
# Each profiled run is bench.py --steps 3 --warmup 1 under hipGraph replay: 1 eager warm-up,
# 1 GraphedStep warm-up, 1 untimed replay, 3 timed replays = 6 training steps of kernels.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=$1; shift
wls=${@:-bisenet-seg bisenet-da deeplab-seg deeplab-da}
# heartbeat: PMC passes print nothing for minutes on the larger workloads
( while sleep 50; do date >> gpurun_out/prof_${tag}_heartbeat; done ) &
hb=$!
trap "kill $hb" EXIT
STEPS=6
for wl in $wls; do
  o=gpurun_out/prof_${tag}_$wl; r=/tmp/prof_${tag}/$wl; mkdir -p $o $r
  args="bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline --no-infer --no-conv-profile --submit branches"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $r/kt -o run -- python3 $args > $o/log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $r/fetch -o run -- python3 $args >> $o/log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $r/write -o run -- python3 $args >> $o/log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $r/mfma -o run -- python3 $args >> $o/log 2>&1
  python3 tools/diag/copy_sites.py $(ls $r/kt/run_kernel_trace.csv) > $o/copy_sites.txt || true
  python3 tools/diag/copy_sites.py $(ls $r/kt/run_kernel_trace.csv) adam_dev_kernel vectorized_elementwise > $o/torch_elementwise_sites.txt || true
  python3 tools/kstats.py $(ls $r/kt/run_kernel_stats.csv) $STEPS > $o/kernel_stats.txt
  python3 tools/kstats.py $(ls $r/kt/run_kernel_stats.csv) $STEPS --all > $o/kernel_stats_all.txt
  python3 tools/pmc_traffic.py $r $STEPS $o/traffic.json > $o/traffic.txt
  python3 tools/pmc_traffic.py $r $STEPS --variants > $o/traffic_by_variant.txt || true
  python3 tools/pmc_mfma_summary.py $(ls $r/mfma/run_counter_collection.csv) $STEPS > $o/mfma.txt
  echo "$wl done"
done
