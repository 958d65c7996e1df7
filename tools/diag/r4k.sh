#!/bin/bash
# image-conv output staging A/B (var_head = HEAD kernels) + tapconv check
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r4k_diag.txt
: > $o
for r in 1 2; do
for lib in var_head librtsds_hip; do
  for a in "fwdstats 8 3 512 1024 64 7 2 3" "eval 8 3 512 1024 64 7 2 3" "pool 8 3 512 1024 64 7 2 3" "fwdstats 8 3 512 1024 64 3 2 1" "eval 8 3 512 1024 64 3 2 1" "fwd 8 64 128 256 64 3 1 1" "dgrad 8 64 128 256 64 3 1 1"; do
    RTSDS_LIB=$PWD/rtsds_amd/$lib.so timeout -k 5 60 python3 tools/diag/time_one.py $a >> $o 2>&1
  done
done
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4k_pytest.log 2>&1 || echo "pytest failed"
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r4k_bench.json 2> gpurun_out/r4k_bench.err
echo ok
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/r4k_kt -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-infer --no-conv-profile --submit branches > gpurun_out/r4k_kt.log 2>&1
python3 tools/diag/copy_sites.py $(ls /tmp/r4k_kt/run_kernel_trace.csv) > gpurun_out/r4k_copy_sites.txt 2>&1 || true
