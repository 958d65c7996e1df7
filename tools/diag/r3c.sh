#!/bin/bash
# graph-split replay + inference fast paths: GPU suite, enqueue diag, bench line, inference profile
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/r3c_pytest.log 2>&1
timeout -k 10 200 python -u tools/diag/enqueue.py > $o/r3c_enq.txt 2>&1
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $o/r3c_bench.json 2> $o/r3c_bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r3c_inf -o run -- python3 tools/diag/infer.py --reps 20 > $o/r3c_infer.log 2>&1
python3 tools/kstats.py $(ls /tmp/r3c_inf/run_kernel_stats.csv) 25 > $o/r3c_infer_kstats.txt
python3 tools/diag/ktrace_seq.py $(ls /tmp/r3c_inf/run_kernel_trace.csv) 110 > $o/r3c_infer_seq.txt
echo ok
