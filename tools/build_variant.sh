#!/bin/bash
# Build an in-tree variant of librtsds_hip.so with extra -D flags (kernel A/B experiments):
#   tools/build_variant.sh NAME "-DFLAG1 -DFLAG2"  ->  rtsds_amd/var_NAME.so
set -e
cd "$(dirname "$0")/../rtsds_amd/csrc"
name=$1; flags=$2
out=build/var_$name
mkdir -p $out
for f in conv hconv imgconv tapconv pw bn ew upce data graph; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Wno-unused-variable $flags -c $f.hip -o $out/$f.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../var_$name.so $out/*.o
echo built rtsds_amd/var_$name.so
