"""Micro-benchmark of the context-path resizes into the fusion module's input (BiSeNet bs 8
1024x512 inference: [8, 256, 32, 64] x2 and [8, 512, 16, 32] x4 -> 64 x 128, channel scales
applied, written into a 1024-channel NHWC buffer; rtsds_bilinear_fwd_scaled) for library A/B:
    RTSDS_LIB=... python tools/bench_resize_cat.py OUT.pt
Saves the output so variants can be compared bit for bit."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rtsds_amd import functional as F  # noqa: E402

dev = "cuda"
g = torch.Generator().manual_seed(5)
CL = torch.channels_last
dt = torch.bfloat16
sx = torch.randn(8, 256, 64, 128, generator=g).to(dev, dt).contiguous(memory_format=CL)
f3 = torch.randn(8, 256, 32, 64, generator=g).to(dev, dt).contiguous(memory_format=CL)
f4 = torch.randn(8, 512, 16, 32, generator=g).to(dev, dt).contiguous(memory_format=CL)
a1 = torch.rand(8, 256, 1, 1, generator=g).to(dev, dt)
a2 = torch.rand(8, 512, 1, 1, generator=g).to(dev, dt)
t = torch.randn(8, 512, 1, 1, generator=g).to(dev, dt)
buf = torch.empty(8, 1024, 64, 128, device=dev, dtype=dt).contiguous(memory_format=CL)
buf[:, :256] = sx
view = buf[:, :256]
run = lambda: F.concat_resized_scaled_eval(view, ((f3, (a1,)), (f4, (a2, t))), (64, 128), into=buf)  # noqa: E731
y = run()
torch.cuda.synchronize()
for r in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(100):
        run()
    e1.record()
    torch.cuda.synchronize()
    print(f"resize x2 (256 ch) + x4 (512 ch) into the concat, bs 8: {e0.elapsed_time(e1) / 100 * 1e3:.1f} us", flush=True)
if len(sys.argv) > 1:
    torch.save(y.cpu(), sys.argv[1])
