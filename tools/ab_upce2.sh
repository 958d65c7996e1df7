#!/bin/bash
# upce.hip variants: bit-level outputs vs the first variant, then fwd+bwd timing (interleaved)
set -e
cd "$GRAFT_REPO_ROOT"
for v in "$@"; do RTSDS_LIB=$PWD/rtsds_amd/var_$v.so timeout -k 10 120 python3 tools/upce_dump.py /tmp/upce_$v.pt 2>/dev/null; done
python3 - "$@" <<'PY'
import sys, torch
vs = sys.argv[1:]
ref = torch.load(f"/tmp/upce_{vs[0]}.pt")
for v in vs[1:]:
    d = torch.load(f"/tmp/upce_{v}.pt")
    same = torch.equal(d["loss"], ref["loss"]) and torch.equal(d["correct"], ref["correct"]) and all(
        torch.equal(a, b) for a, b in zip(d["grads"], ref["grads"]))
    print(f"{v} vs {vs[0]}: bit-identical {same}; loss {d['loss'].item():.6f} / {ref['loss'].item():.6f}")
PY
for r in 1 2; do bash tools/ab_upce.sh "$@"; done
