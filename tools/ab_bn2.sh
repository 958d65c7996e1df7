#!/bin/bash
# BatchNorm backward kernels per variant and shape (kernel-trace averages): ab_bn2.sh base v1 ...
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
shapes=${SHAPES:-"1048576,64 262144,64 262144,128 65536,128 65536,256 16384,256 4096,512"}
for v in "$@"; do
  lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
  for sh in $shapes; do
    RTSDS_LIB=$PWD/$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/abbn2_${v}_${sh}_${BN_FWD:-b}${BN_Y:-} -o run -- python3 tools/bench_bn.py ${sh//,/ } 20 > /dev/null 2>&1 || exit 1
    python3 - /tmp/abbn2_${v}_${sh}_${BN_FWD:-b}${BN_Y:-}/run_kernel_stats.csv "$v $sh" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
out = []
for r in rows:
    n = r["Name"]
    if "bn_" not in n: continue
    short = n.split("(")[0].split("<")[0].replace("_Z19", "").replace("_Z22", "")[:28]
    out.append(f"{short} {float(r['AverageNs'])/1e3:.1f}us")
print(sys.argv[2], " | ".join(sorted(out)))
PY
  done
done
