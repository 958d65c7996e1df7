set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for wl in ${@:-bisenet-seg bisenet-da}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ktq/$wl -o run -- python3 bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline --no-infer --no-conv-profile > gpurun_out/ktq_$wl.log 2>&1
  python3 tools/kstats.py /tmp/ktq/$wl/run_kernel_stats.csv 6 > gpurun_out/ktq_${wl}.txt
done
echo ok
