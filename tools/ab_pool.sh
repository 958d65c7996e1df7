#!/bin/bash
cd "$GRAFT_REPO_ROOT"
for r in 1 2; do for v in ph1 ph2 ph3; do echo "== $v"; RTSDS_LIB=$PWD/rtsds_amd/var_$v.so timeout -k 10 120 python -u tools/bench_imgconv.py 2>&1 | grep -v amdgpu; done; done
