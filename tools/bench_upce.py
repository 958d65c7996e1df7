"""Micro-benchmark of the fused upsample+CE kernels at the BiSeNet bench geometry
(3 heads of [8, 19, 64, 128] bf16 -> 512x1024), for rocprofv3 counter runs."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from rtsds_amd import functional as F

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = "cuda"
heads = [torch.randn(8, 19, 64, 128, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
         .requires_grad_() for _ in range(3)]
t = torch.randint(0, 20, (8, 512, 1024), device=dev)
geo = F.upsample_geometry(heads[0], scale_factor=8)
for i in range(iters):
    if i == 3:
        torch.cuda.synchronize()
        t0 = time.time()
    correct = torch.zeros(1, dtype=torch.int64, device=dev)
    loss = F.upsample_cross_entropy(heads, t, geo, 19, correct)
    loss.backward()
torch.cuda.synchronize()
print(f"upce fwd+bwd: {(time.time() - t0) / (iters - 3) * 1e3:.3f} ms/iter")
