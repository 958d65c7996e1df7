"""Micro-benchmark of the eval forward's final resize (19-class logits x8, BiSeNet bs8
1024x512: [8, 19, 64, 128] -> 512x1024, channels-last) for library A/B runs:
    RTSDS_LIB=... python tools/bench_bilinear.py OUT.pt
Saves the outputs (bf16 and fp32) so variants can be compared bit for bit."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from rtsds_amd import functional as F

dev = "cuda"
g = torch.Generator(device="cpu").manual_seed(3)
out = {}
for dt in (torch.bfloat16, torch.float32):
    x = (torch.randn(8, 19, 64, 128, generator=g) * 3).to(dev, dt).contiguous(memory_format=torch.channels_last)
    geo = F.upsample_geometry(x, scale_factor=8)
    y = F.interpolate_geometry(x, geo)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        F.interpolate_geometry(x, geo)
    e1.record()
    torch.cuda.synchronize()
    print(f"{str(dt):16s} x8 resize 19ch bs8: {e0.elapsed_time(e1) / 50 * 1e3:.1f} us")
    out[str(dt)] = y.cpu()
    # non-integer scale, ragged sizes
    x2 = torch.randn(2, 19, 13, 17, generator=g).to(dev, dt).contiguous(memory_format=torch.channels_last)
    out[str(dt) + "_ragged"] = F.interpolate_geometry(x2, F.upsample_geometry(x2, size=(97, 129))).cpu()
# the context-path resizes of the eval forward (16-B channel vectors, x2 and x4 to 1/8 resolution)
for c, hi, wi in ((256, 32, 64), (512, 16, 32)):
    for dt in (torch.bfloat16,):
        x = torch.randn(8, c, hi, wi, generator=g).to(dev, dt).contiguous(memory_format=torch.channels_last)
        geo = F.upsample_geometry(x, size=(64, 128))
        y = F.interpolate_geometry(x, geo)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            F.interpolate_geometry(x, geo)
        e1.record()
        torch.cuda.synchronize()
        print(f"{str(dt):16s} {c}ch {hi}x{wi} -> 64x128 bs8: {e0.elapsed_time(e1) / 50 * 1e3:.1f} us")
        out[f"{dt}_{c}"] = y.cpu()
        x2 = torch.randn(2, c, 13, 17, generator=g).to(dev, dt).contiguous(memory_format=torch.channels_last)
        out[f"{dt}_{c}_ragged"] = F.interpolate_geometry(x2, F.upsample_geometry(x2, size=(50, 61))).cpu()
if len(sys.argv) > 1:
    torch.save(out, sys.argv[1])
