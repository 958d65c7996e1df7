#!/bin/bash
# bilinear resize variants: timing + bit-level comparison against the first (ab_bilinear.sh base v1 ...)
set -e
cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
  echo "== $v"; RTSDS_LIB=$PWD/$lib timeout -k 10 120 python3 tools/bench_bilinear.py /tmp/bil_$v.pt
done
python3 - "$@" <<'PY'
import sys, torch
vs = sys.argv[1:]
ref = torch.load(f"/tmp/bil_{vs[0]}.pt")
for v in vs[1:]:
    d = torch.load(f"/tmp/bil_{v}.pt")
    print(v, "vs", vs[0], {k: torch.equal(d[k], ref[k]) for k in ref})
PY
