#!/bin/bash
# A/B of kernel units against an older revision: rtsds_amd/var_NAME.so = the listed units from
# git revision REV + every other unit from the current build (make -C rtsds_amd/csrc first), so
# the variant keeps the current ABI revision:  tools/build_unit_rev.sh NAME REV UNIT [UNIT ...]
set -e
cd "$(dirname "$0")/../rtsds_amd/csrc"
name=$1; rev=$2; shift 2
out=build/unitrev_$name
rm -rf $out && mkdir -p $out
trap 'rm -f _rev_*.hip' EXIT
for unit in "$@"; do
  git show $rev:rtsds_amd/csrc/$unit.hip > _rev_$unit.hip
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function -Wno-unused-variable -c _rev_$unit.hip -o $out/$unit.o &
done
wait
for f in build/*.o; do [ -e $out/$(basename $f) ] || cp $f $out/; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../var_$name.so $out/*.o
echo built rtsds_amd/var_$name.so: "$@" from $rev
