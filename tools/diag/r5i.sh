#!/bin/bash
# Mid-round evidence (r5a): bench default line, rocprofv3 kernel trace + FETCH/WRITE + MFMA passes
# of the bisenet-seg and deeplab-seg workloads and of the bs-8 inference forward.
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python3 bench.py > gpurun_out/r5a_bench_default.json 2> gpurun_out/r5a_bench_default.err || exit 1
head -c 400 gpurun_out/r5a_bench_default.json; echo
timeout -k 10 1200 bash tools/profile_all.sh r5a bisenet-seg deeplab-seg || exit 1
timeout -k 10 600 bash tools/profile_infer.sh r5a || exit 1
echo done
