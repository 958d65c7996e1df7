set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in base big1 big2 big3; do
  lib=""; [ $v != base ] && lib=rtsds_amd/var_$v.so
  bash tools/conv_suite.sh $lib > gpurun_out/big_$v.log 2>&1
  echo "$v done"
done
