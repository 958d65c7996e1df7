#!/bin/bash
# Iteration check: a GPU test selection (-k expression), the headline bench line (no CPU
# baseline) and a kernel-trace summary of it.  usage: quick_check.sh TAG "KEXPR" [bench args]
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=$1; kexpr=$2; shift 2 || true
if [ -n "$kexpr" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$kexpr" > gpurun_out/${tag}_pytest.log 2>&1
fi
timeout -k 10 400 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_${tag} -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-infer --no-conv-profile "$@" > gpurun_out/${tag}_prof.log 2>&1
python3 tools/kstats.py /tmp/prof_${tag}/run_kernel_stats.csv 15 > gpurun_out/${tag}_kernel_stats.txt
echo done
