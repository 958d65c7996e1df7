#!/bin/bash
# Full GPU check: gpu tests, smoke, bench, rocprof kernel-trace summary. Outputs under gpurun_out/.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-check}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_${tag} -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-infer > gpurun_out/${tag}_prof.log 2>&1
python3 tools/kstats.py /tmp/prof_${tag}/run_kernel_stats.csv 15 > gpurun_out/${tag}_kernel_stats.txt
echo done
