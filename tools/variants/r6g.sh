#!/bin/bash
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 bash tools/variants/pmc_conv_ceiling.sh r6g > gpurun_out/r6g_conv_ceiling.txt 2>&1 || exit 1
timeout -k 10 900 bash tools/profile_all.sh r6g bisenet-seg > gpurun_out/r6g_prof.log 2>&1 || exit 1
timeout -k 10 600 bash tools/profile_infer.sh r6g >> gpurun_out/r6g_prof.log 2>&1
