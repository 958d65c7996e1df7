#!/bin/bash
cd "$GRAFT_REPO_ROOT"
for r in 1 2; do for v in base bilu1 bilu4; do
  lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
  echo "== $v"; RTSDS_LIB=$PWD/$lib timeout -k 10 120 python3 tools/bench_resize_cat.py /tmp/rc_$v.pt 2>&1 | grep -v amdgpu || exit 1
done; done > gpurun_out/r6f_resize.txt
python3 -c "
import torch; r = torch.load('/tmp/rc_base.pt')
for v in ('bilu1', 'bilu4'): print(v, 'bit-identical to base:', torch.equal(torch.load(f'/tmp/rc_{v}.pt'), r))" >> gpurun_out/r6f_resize.txt
for r in 1 2; do for v in base bilu1 bilu4; do
  lib=rtsds_amd/var_$v.so; [ "$v" = base ] && lib=rtsds_amd/librtsds_hip.so
  echo -n "$v "; RTSDS_LIB=$PWD/$lib timeout -k 10 120 python3 tools/diag/infer.py --batch 8 --reps 300 2>&1 | grep -v amdgpu || exit 1
done; done > gpurun_out/r6f_infer.txt
