#!/bin/bash
# session-2 iteration: upce variant A/B, focused GPU tests, the headline bench + kernel stats
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=$1
bash tools/ab_upce2.sh upold up2 > gpurun_out/${tag}_ab_upce.txt 2>&1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "image_conv or padded_image or stem or conv_fwd_bwd or upsample_cross or upce or fused or dgrad_epilogue or branch_streams or bisenet" > gpurun_out/${tag}_pytest.log 2>&1
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_${tag} -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-infer --no-conv-profile > gpurun_out/${tag}_prof.log 2>&1
python3 tools/kstats.py /tmp/prof_${tag}/run_kernel_stats.csv 15 > gpurun_out/${tag}_kernel_stats.txt
echo done
