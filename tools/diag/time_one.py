"""Time one conv pass (HIP events around `iters` back-to-back launches).  usage: time_one.py PASS N C H W K KH STRIDE PAD [iters]"""
import ctypes, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from rtsds_amd import functional as F  # noqa: E402
from rtsds_amd._lib import lib  # noqa: E402
from rtsds_amd.runtime import workspace  # noqa: E402
pas = sys.argv[1]
n, c, h, w, k, kh, s, p = [int(v) for v in sys.argv[2:10]]
iters = int(sys.argv[10]) if len(sys.argv) > 10 else 50
dev = "cuda"
CL = torch.channels_last
x = torch.randn(n, c, h, w, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)
wt = (torch.randn(k, c, kh, kh, device=dev) * 0.05).to(torch.bfloat16).contiguous(memory_format=CL)
d = F._conv_desc(x, k, kh, kh, (s, s), (p, p), (1, 1))
y = torch.empty(n, k, d.ho, d.wo, device=dev, dtype=torch.bfloat16).contiguous(memory_format=CL)
dy = torch.randn_like(y)
dx = torch.empty_like(x)
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
st = torch.cuda.current_stream().cuda_stream
wsf = workspace(lib.rtsds_conv2d_fwd_workspace(ctypes.byref(d)), x.device)
wsd = workspace(lib.rtsds_conv2d_dgrad_workspace(ctypes.byref(d)), x.device)
wsw = workspace(lib.rtsds_conv2d_wgrad_workspace(ctypes.byref(d)), x.device)
dw, db = torch.empty(k, c * kh * kh, device=dev), torch.empty(k, device=dev)
sp = torch.empty(k * max(1, lib.rtsds_conv2d_fwd_stats_tiles(ctypes.byref(d))) * 4, device=dev)
sc, sh = torch.ones(k, device=dev), torch.zeros(k, device=dev)
hp, wp = (d.ho + 2 - 3) // 2 + 1, (d.wo + 2 - 3) // 2 + 1
yp = torch.empty(n, k, hp, wp, device=dev, dtype=torch.bfloat16).contiguous(memory_format=CL)
# 3-channel images: the network hands the convs the 4-channel padded image (RTSDS_INPUT_PADDED,
# functional.pack_input), so time the kernels on that (no pad pass inside the timed call)
pad = 0
if c == 3 and os.environ.get("TIME_ONE_UNPADDED") is None:
    x = torch.nn.functional.pad(x.permute(0, 2, 3, 1), (0, 1)).contiguous()
    pad = 0x400
fn = {"fwd": lambda: lib.rtsds_conv2d_fwd(ctypes.byref(d), P(x), P(wt), None, P(y), pad, None, P(wsf), wsf.numel(), st),
      "fwdstats": lambda: lib.rtsds_conv2d_fwd(ctypes.byref(d), P(x), P(wt), None, P(y), pad, P(sp), P(wsf), wsf.numel(), st),
      "eval": lambda: lib.rtsds_conv2d_fwd_bn(ctypes.byref(d), P(x), P(wt), P(sc), P(sh), None, P(y), 1 | pad, P(wsf), wsf.numel(), st),
      "pool": lambda: lib.rtsds_conv2d_fwd_bn_maxpool(ctypes.byref(d), P(x), P(wt), P(sc), P(sh), P(yp), 1 | pad, hp, wp, 1,
                                                      P(wsf), wsf.numel(), st),
      "dgrad": lambda: lib.rtsds_conv2d_dgrad(ctypes.byref(d), P(dy), P(wt), P(dx), 0, P(wsd), wsd.numel(), st),
      "wgrad": lambda: lib.rtsds_conv2d_wgrad(ctypes.byref(d), P(x), P(dy), P(dw), P(db), pad, P(wsw), wsw.numel(), st)}[pas]
for _ in range(5):
    fn()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(iters):
    fn()
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1000 / iters
print(f"{os.path.basename(os.environ.get('RTSDS_LIB', 'librtsds_hip.so')):24s} {pas} {' '.join(sys.argv[2:10])}: {us:7.1f} us  {2.0 * n * d.ho * d.wo * k * c * kh * kh / us / 1e6:7.1f} TF/s", flush=True)
