#!/bin/bash
# round-3 diagnostics: graph-launch host cost under HIP graph env settings, ordered kernel
# trace of the seg step, inference-forward kernel profile
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out
timeout -k 10 200 python -u tools/diag/enqueue.py > $o/r3b_enq_default.txt 2>&1
DEBUG_HIP_FORCE_GRAPH_QUEUES=1 timeout -k 10 200 python -u tools/diag/enqueue.py > $o/r3b_enq_q1.txt 2>&1
DEBUG_HIP_FORCE_GRAPH_QUEUES=2 timeout -k 10 200 python -u tools/diag/enqueue.py > $o/r3b_enq_q2.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/r3b_kt -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-infer --no-conv-profile > $o/r3b_kt.log 2>&1
python3 tools/diag/ktrace_seq.py $(ls /tmp/r3b_kt/run_kernel_trace.csv) 500 > $o/r3b_seq.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r3b_inf -o run -- python3 tools/diag/infer.py --reps 20 > $o/r3b_infer.log 2>&1
python3 tools/kstats.py $(ls /tmp/r3b_inf/run_kernel_stats.csv) 25 > $o/r3b_infer_kstats.txt
python3 tools/diag/ktrace_seq.py $(ls /tmp/r3b_inf/run_kernel_trace.csv) 120 > $o/r3b_infer_seq.txt
timeout -k 10 120 python -u tools/diag/infer.py --reps 50 > $o/r3b_infer_plain.txt 2>&1
echo ok
