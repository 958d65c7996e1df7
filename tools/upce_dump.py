"""Fused upsample + CE at the BiSeNet bench geometry on fixed seeded inputs: saves the loss,
accuracy count and head gradients (bit-level A/B of upce.hip variants).  usage: upce_dump.py OUT"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rtsds_amd import functional as F  # noqa: E402

g = torch.Generator(device="cuda").manual_seed(3)
heads = [(torch.randn(8, 19, 64, 128, device="cuda", generator=g) * 3).to(torch.bfloat16)
         .contiguous(memory_format=torch.channels_last).requires_grad_() for _ in range(3)]
t = torch.randint(0, 20, (8, 512, 1024), device="cuda", generator=g)
geo = F.upsample_geometry(heads[0], scale_factor=8)
correct = torch.zeros(1, dtype=torch.int64, device="cuda")
loss = F.upsample_cross_entropy(heads, t, geo, 19, correct)
loss.backward()
torch.save({"loss": loss.detach().cpu(), "correct": correct.cpu(), "grads": [h.grad.float().cpu() for h in heads]},
           sys.argv[1])
