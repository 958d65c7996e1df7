#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -x -q --timeout 200 --timeout-method thread -k "inference_fast_path" > $o/r3e_pytest.log 2>&1
timeout -k 10 60 ./tools/probe/last_arriver > $o/r3e_last_arriver.txt 2>&1
timeout -k 10 300 python -u tools/diag/enqueue.py --modes branches+split2,branches+split3,branches,serial > $o/r3e_enq.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r3e_inf -o run -- python3 tools/diag/infer.py --reps 20 > $o/r3e_infer.log 2>&1
python3 tools/kstats.py $(ls /tmp/r3e_inf/run_kernel_stats.csv) 25 > $o/r3e_infer_kstats.txt
timeout -k 10 120 python -u tools/diag/infer.py --reps 50 > $o/r3e_infer_plain.txt 2>&1
echo ok
