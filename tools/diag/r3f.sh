#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/r3f_pytest.log 2>&1
timeout -k 10 300 python -u tools/diag/enqueue.py > $o/r3f_enq.txt 2>&1
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $o/r3f_bench.json 2> $o/r3f_bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r3f_kt -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-infer --no-conv-profile > $o/r3f_kt.log 2>&1
python3 tools/kstats.py $(ls /tmp/r3f_kt/run_kernel_stats.csv) 9 > $o/r3f_kstats.txt
echo ok
