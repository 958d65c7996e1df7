set -e
cd "$GRAFT_REPO_ROOT"
for r in 1 2; do for v in a11 a22 a24 a12; do echo "== $v"; RTSDS_LIB=$PWD/rtsds_amd/var_$v.so timeout -k 10 120 python -u tools/bench_imgconv.py; done; done > gpurun_out/ab_img.txt 2>&1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "image_conv or padded_image or stem or conv_fwd_bwd" > gpurun_out/ab_img_pytest.log 2>&1
echo done
