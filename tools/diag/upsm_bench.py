"""Fused upsample-softmax forward + backward at the DA bench geometry (8 x 19 x 64 x 128 ->
512 x 1024, bf16), for rocprofv3 kernel / counter runs."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

import rtsds_amd
from rtsds_amd import functional as F

rtsds_amd.set_compute_dtype(torch.bfloat16)
x = torch.randn(8, 19, 64, 128, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
x.requires_grad_()
geo = F.upsample_geometry(x, size=(512, 1024))
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 10):
    y = F.upsample_softmax(x, geo)
    y.backward(torch.ones_like(y))
torch.cuda.synchronize()
print("ok")
