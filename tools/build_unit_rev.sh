#!/bin/bash
# A/B of kernel units against an older revision: rtsds_amd/var_NAME.so = the listed units (and
# the csrc headers) from git revision REV + every other unit from the current build (make -C
# rtsds_amd/csrc first); the C ABI header is the current one, so the variant keeps the current
# ABI revision:  tools/build_unit_rev.sh NAME REV UNIT [UNIT ...]
set -e
root="$(cd "$(dirname "$0")/.." && pwd)"
cd "$root"
name=$1; rev=$2; shift 2
# the conv host side (conv.hip) and the GEMM kernel units share conv_args.h (the tile choice,
# which also sizes the BatchNorm-statistics partials): swapping one without the others mixes two
# tile rules -- a launch then writes partials for more M tiles than its caller allocated (a GPU
# memory fault, round 5).  They always travel together.
units=" $* "
if [[ "$units" =~ " conv " || "$units" == *" conv_gemm_"* ]]; then
  for u in conv conv_gemm_fwd conv_gemm_dgrad conv_gemm_wgrad; do
    git cat-file -e $rev:rtsds_amd/csrc/$u.hip 2>/dev/null && [[ "$units" != *" $u "* ]] && units="$units$u "
  done
fi
set -- $units
src=_revtmp/src   # two levels below the root: the sources' ../../include/rtsds_hip.h resolves
out=rtsds_amd/csrc/build/unitrev_$name
rm -rf _revtmp $out && mkdir -p $src $out
trap 'rm -rf "$root/_revtmp"' EXIT
for h in $(git ls-tree --name-only $rev rtsds_amd/csrc/ | grep -E '\.h$'); do git show $rev:$h > $src/$(basename $h); done
for unit in "$@"; do
  git show $rev:rtsds_amd/csrc/$unit.hip > $src/$unit.hip
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function -Wno-unused-variable -c $src/$unit.hip -o $out/$unit.o &
done
wait
for f in rtsds_amd/csrc/build/*.o; do [ -e $out/$(basename $f) ] || cp $f $out/; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o rtsds_amd/var_$name.so $out/*.o
echo built rtsds_amd/var_$name.so: "$@" from $rev
