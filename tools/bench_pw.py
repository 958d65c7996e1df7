"""Event-timed narrow 1x1 data gradient (pw.hip) at the BiSeNet supervision heads' shapes, fresh
and accumulating: python3 tools/bench_pw.py (RTSDS_LIB selects a variant build)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rtsds_amd._lib import lib  # noqa: E402
from rtsds_amd.functional import _P, _conv_desc  # noqa: E402
from rtsds_amd.runtime import stream, workspace  # noqa: E402

dev = torch.device("cuda")
for n, c, h, w in ((8, 256, 32, 64), (8, 512, 16, 32), (8, 19, 64, 128)):
    k = 19
    x = torch.randn(n, c, h, w, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(n, k, h, w, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wq = (torch.randn(k, c, 1, 1, device=dev) / c ** 0.5).to(torch.bfloat16)
    d = _conv_desc(x, k, 1, 1, (1, 1), (0, 0), (1, 1))
    dx = torch.empty_like(x)
    ws = workspace(lib.rtsds_conv2d_dgrad_workspace(ctypes.byref(d)), dev)
    for acc in (0, 1):
        for _ in range(20):
            lib.rtsds_conv2d_dgrad(ctypes.byref(d), _P(dy), _P(wq), _P(dx), acc, _P(ws), ws.numel(), stream())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(200):
            lib.rtsds_conv2d_dgrad(ctypes.byref(d), _P(dy), _P(wq), _P(dx), acc, _P(ws), ws.numel(), stream())
        e1.record()
        torch.cuda.synchronize()
        print(f"{os.environ.get('RTSDS_LIB', 'base').split('/')[-1]:24s} {n}x{c}x{h}x{w} -> {k} accumulate {acc}: "
              f"{e0.elapsed_time(e1) / 200 * 1000:.1f} us", flush=True)
