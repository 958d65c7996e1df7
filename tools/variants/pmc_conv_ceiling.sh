#!/bin/bash
# MFMA-busy / wait counters of the shipped conv kernels against the bare K loop
# (tools/variants/conv_diag_variant.py both) on BiSeNet layer shapes: pmc_conv_ceiling.sh TAG
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=$1
for v in base diag_both; do
  lib=$PWD/rtsds_amd/var_$v.so; [ "$v" = base ] && lib=$PWD/rtsds_amd/librtsds_hip.so
  for sh in "8 128 64 128 128 3 1 1" "8 64 256 512 128 3 2 1"; do
    d=/tmp/pmcc_${tag}_${v}_${sh// /_}
    RTSDS_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $d -o run -- python3 tools/bench_conv.py $sh 5 > /dev/null 2>&1
    echo "== $v $sh"
    python3 tools/pmc_mfma_summary.py $(ls $d/run_counter_collection.csv) 1 | grep -E "kernel|conv_gemm" | head -8
  done
done
