#!/bin/bash
# Build rtsds_amd/var_NAME.so from the kernel sources of git revision REV (A/B against the
# working tree):  tools/build_rev_variant.sh NAME REV
set -e
cd "$(dirname "$0")/.."
name=$1; rev=${2:-HEAD}
tmp=rtsds_amd/csrc/build/rev_$name
rm -rf $tmp && mkdir -p $tmp/x/src $tmp/include $tmp/obj   # (common.h includes ../../include/rtsds_hip.h)
git show $rev:include/rtsds_hip.h > $tmp/include/rtsds_hip.h
for f in $(git ls-tree --name-only $rev rtsds_amd/csrc/ | grep -E '\.(hip|h)$'); do git show $rev:$f > $tmp/x/src/$(basename $f); done
srcs=$(cd $tmp/x/src && ls *.hip)
for f in $srcs; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function -Wno-unused-variable -c $tmp/x/src/$f -o $tmp/obj/${f%.hip}.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o rtsds_amd/var_$name.so $tmp/obj/*.o
echo built rtsds_amd/var_$name.so from $rev
