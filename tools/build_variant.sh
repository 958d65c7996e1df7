#!/bin/bash
# Build an in-tree variant of librtsds_hip.so with extra -D flags (kernel A/B experiments):
#   tools/build_variant.sh NAME "-DFLAG1 -DFLAG2" [units]  ->  rtsds_amd/var_NAME.so
# units (e.g. "bn ew"): only these .hip files are recompiled with the flags; the others are
# linked from the main build's objects (make -C rtsds_amd/csrc first).  Default: all units.
set -e
cd "$(dirname "$0")/../rtsds_amd/csrc"
name=$1; flags=$2; units=${3:-"conv conv_gemm_fwd conv_gemm_dgrad conv_gemm_wgrad hconv imgconv tapconv pw bn ew upce data graph"}
out=build/var_$name
rm -rf $out && mkdir -p $out
for f in conv conv_gemm_fwd conv_gemm_dgrad conv_gemm_wgrad hconv imgconv tapconv pw bn ew upce data graph; do
  if [[ " $units " == *" $f "* ]]; then
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Wno-unused-variable $flags -c $f.hip -o $out/$f.o &
  else
    cp build/$f.o $out/$f.o
  fi
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../var_$name.so $out/*.o
echo built rtsds_amd/var_$name.so
