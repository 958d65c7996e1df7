"""Times the 3-channel stride-2 image convs (imgconv.hip) at the bench geometries through the C
ABI: forward with the BatchNorm-statistics epilogue (train) and the eval BN fold + ReLU, for the
ResNet stem (7x7 s2 p3) and the spatial-path conv (3x3 s2 p1), input in the 4-channel pitch
(pack_input).  usage: bench_imgconv.py [N H W] [iters]"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rtsds_amd import functional as F  # noqa: E402
from rtsds_amd._lib import INPUT_PADDED, lib  # noqa: E402
from rtsds_amd.runtime import workspace  # noqa: E402

n, h, w = [int(v) for v in sys.argv[1:4]] if len(sys.argv) > 3 else (8, 512, 1024)
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 50
dev = "cuda"
CL = torch.channels_last
P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
st = torch.cuda.current_stream().cuda_stream
x = F.pack_input(torch.randn(n, 3, h, w, device=dev) * 50, torch.bfloat16)
for kh, pad in ((7, 3), (3, 1)):
    wt = (torch.randn(64, 3, kh, kh, device=dev) * 0.05).to(torch.bfloat16).contiguous(memory_format=CL)
    d = F._conv_desc(x, 64, kh, kh, (2, 2), (pad, pad), (1, 1))
    y = torch.empty(n, 64, d.ho, d.wo, device=dev, dtype=torch.bfloat16).contiguous(memory_format=CL)
    nrb = lib.rtsds_conv2d_fwd_stats_tiles(ctypes.byref(d))
    stats = torch.empty(nrb * 64 * 4, device=dev)
    ss = torch.rand(128, device=dev)
    ws = workspace(lib.rtsds_conv2d_fwd_workspace(ctypes.byref(d)), x.device)
    runs = (("train+stats", lambda: lib.rtsds_conv2d_fwd(ctypes.byref(d), P(x), P(wt), None, P(y), INPUT_PADDED, P(stats),
                                                         P(ws), ws.numel(), st)),
            ("eval fold+relu", lambda: lib.rtsds_conv2d_fwd_bn(ctypes.byref(d), P(x), P(wt), P(ss), ss.data_ptr() + 256, None,
                                                               P(y), 1 | INPUT_PADDED, P(ws), ws.numel(), st)))
    for name, fn in runs:
        for _ in range(5):
            assert fn() == 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / iters
        mb = (x.numel() // 3 * 4 * 2 + y.numel() * 2) / 1e6
        print(f"k{kh} {name:15s} {us:7.1f} us  {mb / us:6.2f} TB/s (input + output {mb:.0f} MB)", flush=True)
# the inference stem with the pool in its epilogue (rtsds_conv2d_fwd_bn_maxpool), bs / size as above
wt = (torch.randn(64, 3, 7, 7, device=dev) * 0.05).to(torch.bfloat16).contiguous(memory_format=CL)
d = F._conv_desc(x, 64, 7, 7, (2, 2), (3, 3), (1, 1))
hp, wp = F.pool_out(d.ho, 3, 2, 1, False), F.pool_out(d.wo, 3, 2, 1, False)
yp = torch.empty(n, 64, hp, wp, device=dev, dtype=torch.bfloat16).contiguous(memory_format=CL)
ss = torch.rand(128, device=dev)
ws = workspace(lib.rtsds_conv2d_fwd_workspace(ctypes.byref(d)), x.device)
fn = lambda: lib.rtsds_conv2d_fwd_bn_maxpool(ctypes.byref(d), P(x), P(wt), P(ss), ss.data_ptr() + 256, P(yp),  # noqa: E731
                                             1 | INPUT_PADDED, hp, wp, 1, P(ws), ws.numel(), st)
for _ in range(5):
    fn()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(iters):
    fn()
e1.record()
torch.cuda.synchronize()
print(f"k7 eval stem+pool  {e0.elapsed_time(e1) * 1e3 / iters:7.1f} us", flush=True)
