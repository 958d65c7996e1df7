"""Run one conv pass (fwd / dgrad / wgrad) of one geometry `iters` times through the C ABI, for
rocprofv3 passes.  usage: conv_one.py PASS N C H W K KH STRIDE PAD [iters] [stats]"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from rtsds_amd import functional as F  # noqa: E402
from rtsds_amd._lib import lib  # noqa: E402
from rtsds_amd.runtime import workspace  # noqa: E402

pas = sys.argv[1]
n, c, h, w, k, kh, s, p = [int(v) for v in sys.argv[2:10]]
iters = int(sys.argv[10]) if len(sys.argv) > 10 else 20
stats = len(sys.argv) > 11 and sys.argv[11] == "stats"
dev = "cuda"
CL = torch.channels_last
x = torch.randn(n, c, h, w, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)
wt = (torch.randn(k, c, kh, kh, device=dev) * 0.05).to(torch.bfloat16).contiguous(memory_format=CL)
d = F._conv_desc(x, k, kh, kh, (s, s), (p, p), (1, 1))
y = torch.empty(n, k, d.ho, d.wo, device=dev, dtype=torch.bfloat16).contiguous(memory_format=CL)
dy = torch.randn_like(y)
dx = torch.empty_like(x)
dw = torch.empty(k, kh, kh, c, device=dev, dtype=torch.float32)
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
st = torch.cuda.current_stream().cuda_stream
wsf = workspace(lib.rtsds_conv2d_fwd_workspace(ctypes.byref(d)), x.device)
wsd = workspace(lib.rtsds_conv2d_dgrad_workspace(ctypes.byref(d)), x.device)
wsw = workspace(lib.rtsds_conv2d_wgrad_workspace(ctypes.byref(d)), x.device)
sp = torch.empty(k * max(1, lib.rtsds_conv2d_fwd_stats_tiles(ctypes.byref(d))) * 4, device=dev) if stats else None
fns = {"fwd": lambda: lib.rtsds_conv2d_fwd(ctypes.byref(d), P(x), P(wt), None, P(y), 0, P(sp) if stats else None, P(wsf), wsf.numel(), st),
       "dgrad": lambda: lib.rtsds_conv2d_dgrad(ctypes.byref(d), P(dy), P(wt), P(dx), 0, P(wsd), wsd.numel(), st),
       "wgrad": lambda: lib.rtsds_conv2d_wgrad(ctypes.byref(d), P(x), P(dy), P(dw), None, 0, P(wsw), wsw.numel(), st)}
for _ in range(iters):
    fns[pas]()
torch.cuda.synchronize()
print("ok")
