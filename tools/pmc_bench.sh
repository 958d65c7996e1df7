#!/bin/bash
# HBM traffic of the bench's kernels: two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; the
# TCC block cannot hold both) over a short bench run -> gpurun_out/pmc_bench_$1/{fetch,write}.
# Summarise with tools/pmc_traffic.py DIR auto (applies the gfx950 FETCH_SIZE x2 correction).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=${1:-r1}; steps=${2:-2}
args="bench.py --steps $steps --warmup 1 --no-cpu-baseline --no-infer --no-conv-profile"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_bench_$tag/fetch -o run -- python3 $args > gpurun_out/pmc_bench_$tag.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_bench_$tag/write -o run -- python3 $args >> gpurun_out/pmc_bench_$tag.log 2>&1
# per-step division: tools/pmc_traffic.py DIR auto (counts the profiled training steps)
