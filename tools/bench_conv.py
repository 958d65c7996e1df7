"""Micro-benchmark of one conv layer (fwd + dgrad + wgrad through the HIP ABI) for
rocprofv3 counter runs.  usage: bench_conv.py N C H W K KH STRIDE PAD [iters] [dilation]"""
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rtsds_amd import functional as F  # noqa: E402
from rtsds_amd._lib import lib  # noqa: E402
from rtsds_amd.runtime import workspace  # noqa: E402

n, c, h, w, k, kh, s, p = [int(v) for v in sys.argv[1:9]]
iters = int(sys.argv[9]) if len(sys.argv) > 9 else 20
dil = int(sys.argv[10]) if len(sys.argv) > 10 else 1
dev = "cuda"
CL = torch.channels_last
x = torch.randn(n, c, h, w, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)
wt = (torch.randn(k, c, kh, kh, device=dev) * 0.05).to(torch.bfloat16).contiguous(memory_format=CL)
d = F._conv_desc(x, k, kh, kh, (s, s), (p, p), (dil, dil))
y = torch.empty(n, k, d.ho, d.wo, device=dev, dtype=torch.bfloat16).contiguous(memory_format=CL)
dy = torch.randn_like(y)
dx = torch.empty_like(x)
dw = torch.empty(k, kh, kh, c, device=dev, dtype=torch.float32)
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
st = torch.cuda.current_stream().cuda_stream
wsf = workspace(lib.rtsds_conv2d_fwd_workspace(ctypes.byref(d)), x.device)
wsd = workspace(lib.rtsds_conv2d_dgrad_workspace(ctypes.byref(d)), x.device)
wsw = workspace(lib.rtsds_conv2d_wgrad_workspace(ctypes.byref(d)), x.device)
flop = 2.0 * n * d.ho * d.wo * k * c * kh * kh
for name, fn in (
        ("fwd", lambda: lib.rtsds_conv2d_fwd(ctypes.byref(d), P(x), P(wt), None, P(y), 0, None, P(wsf), wsf.numel(), st)),
        ("dgrad", lambda: lib.rtsds_conv2d_dgrad(ctypes.byref(d), P(dy), P(wt), P(dx), 0, P(wsd), wsd.numel(), st)),
        ("wgrad", lambda: lib.rtsds_conv2d_wgrad(ctypes.byref(d), P(x), P(dy), P(dw), None, 0, P(wsw), wsw.numel(), st))):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / iters
    print(f"{' '.join(sys.argv[1:9])} d{dil} {name:5s} {dt * 1e6:8.1f} us  {flop / dt / 1e12:7.1f} TF/s", flush=True)
