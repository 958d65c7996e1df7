set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for lib in rtsds_amd/librtsds_hip.so rtsds_amd/var_wg1.so rtsds_amd/var_wg2.so rtsds_amd/librtsds_hip.so; do
  echo "== $lib" >> gpurun_out/wg_ab.log
  for a in "8 3 512 1024 64 3 2 1 20" "8 3 512 1024 64 7 2 3 20" "8 1024 64 128 19 3 1 1 20" "8 64 128 256 64 3 1 1 20" "8 64 256 512 128 3 2 1 20" "8 128 64 128 128 3 1 1 20" "8 256 32 64 256 3 1 1 20" "8 512 16 32 512 3 1 1 20" "8 512 64 128 19 1 1 0 20"; do
    RTSDS_LIB=$lib timeout -k 5 60 python3 tools/bench_conv.py $a 2>/dev/null | grep wgrad >> gpurun_out/wg_ab.log
  done
done
echo ok
