"""Forward conv with and without the BatchNorm-statistics epilogue (the cost of the fused
statistics), interleaved rounds.  usage: bench_conv_stats.py N C H W K KH STRIDE PAD [iters] [dil]"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rtsds_amd import functional as F  # noqa: E402
from rtsds_amd._lib import lib  # noqa: E402
from rtsds_amd.runtime import workspace  # noqa: E402

n, c, h, w, k, kh, s, p = [int(v) for v in sys.argv[1:9]]
iters = int(sys.argv[9]) if len(sys.argv) > 9 else 30
dil = int(sys.argv[10]) if len(sys.argv) > 10 else 1
dev = "cuda"
CL = torch.channels_last
x = torch.randn(n, c, h, w, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)
wt = (torch.randn(k, c, kh, kh, device=dev) * 0.05).to(torch.bfloat16).contiguous(memory_format=CL)
d = F._conv_desc(x, k, kh, kh, (s, s), (p, p), (dil, dil))
y = torch.empty(n, k, d.ho, d.wo, device=dev, dtype=torch.bfloat16).contiguous(memory_format=CL)
nrb = lib.rtsds_conv2d_fwd_stats_tiles(ctypes.byref(d))
stats = torch.empty(nrb * k * 4, device=dev)
P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
st = torch.cuda.current_stream().cuda_stream
ws = workspace(lib.rtsds_conv2d_fwd_workspace(ctypes.byref(d)), x.device)
res = {}
for r in range(3):
    for name, sp in (("plain", None), ("stats", stats)):
        fn = lambda: lib.rtsds_conv2d_fwd(ctypes.byref(d), P(x), P(wt), None, P(y), 0, P(sp), P(ws), ws.numel(), st)  # noqa: E731
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res.setdefault(name, []).append(e0.elapsed_time(e1) * 1e3 / iters)
print(f"{' '.join(sys.argv[1:9])} d{dil}: plain {min(res['plain']):6.1f} us, +stats {min(res['stats']):6.1f} us (nrb {nrb})", flush=True)
