#!/bin/bash
# split-replay trace + inference kernels after the bilinear / FFM-head changes
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -x -q --timeout 200 --timeout-method thread -k "inference_fast_path or graphed_step_equals_eager or bisenet" > $o/r3d_pytest.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 200 --timeout-method thread -k "bilinear or graph" > $o/r3d_pytest_ops.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/r3d_kt -o run -- python3 tools/diag/enqueue.py --modes branches+split --steps 12 > $o/r3d_kt.log 2>&1
python3 tools/diag/ktrace_seq.py $(ls /tmp/r3d_kt/run_kernel_trace.csv) 700 > $o/r3d_split_seq.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r3d_inf -o run -- python3 tools/diag/infer.py --reps 20 > $o/r3d_infer.log 2>&1
python3 tools/kstats.py $(ls /tmp/r3d_inf/run_kernel_stats.csv) 25 > $o/r3d_infer_kstats.txt
python3 tools/diag/ktrace_seq.py $(ls /tmp/r3d_inf/run_kernel_trace.csv) 110 > $o/r3d_infer_seq.txt
timeout -k 10 120 python -u tools/diag/infer.py --reps 50 > $o/r3d_infer_plain.txt 2>&1
timeout -k 10 120 python -u tools/diag/infer.py --reps 200 --batch 1 >> $o/r3d_infer_plain.txt 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 200 > $o/r3d_bench.json 2> $o/r3d_bench.err
timeout -k 10 60 ./tools/probe/last_arriver > $o/r3d_last_arriver.txt 2>&1
bash tools/ab_ring.sh rtsds_amd/librtsds_hip.so rtsds_amd/var_ring3.so rtsds_amd/var_ring4.so > $o/r3d_ring_ab.txt 2>&1
echo ok
