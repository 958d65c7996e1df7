set -e
cd "$GRAFT_REPO_ROOT"
for r in 1 2; do for v in st2 base; do echo "== $v"; lib=$PWD/rtsds_amd/var_$v.so; [ $v = base ] && lib=$PWD/rtsds_amd/librtsds_hip.so; bash tools/conv_stats_suite.sh $lib; done; done > gpurun_out/ab_stats.txt 2>&1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "stats or conv_bn or bisenet_1024 or deeplab or image_conv or stem" > gpurun_out/ab_stats_pytest.log 2>&1
echo done
