"""Micro-benchmark of the BatchNorm backward (stats + finalize + apply) through the HIP ABI,
for kernel-trace A/B runs: bench_bn.py ROWS C [iters]  (bf16, ReLU mask from x)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rtsds_amd._lib import lib  # noqa: E402
from rtsds_amd.runtime import workspace  # noqa: E402

rows, c = int(sys.argv[1]), int(sys.argv[2])
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 20
dev = "cuda"
dy = torch.randn(rows, c, device=dev).to(torch.bfloat16)
x = torch.randn(rows, c, device=dev).to(torch.bfloat16)
dx = torch.empty_like(x)
g = torch.ones(c, device=dev)
b = torch.zeros(c, device=dev)
sm = torch.zeros(c, device=dev)
si = torch.ones(c, device=dev)
dg = torch.empty(c, device=dev)
db = torch.empty(c, device=dev)
ws = workspace(lib.rtsds_bn_workspace(rows, c), x.device)
P = lambda t: t.data_ptr()  # noqa: E731
st = torch.cuda.current_stream().cuda_stream
if os.environ.get("BN_FWD"):  # forward: statistics + finalize + apply (training, ReLU)
    rm, rv, y = torch.zeros(c, device=dev), torch.ones(c, device=dev), torch.empty_like(x)
    fwd = lambda: lib.rtsds_bn_fwd(P(x), None, P(y), rows, c, P(g), P(b), P(rm), P(rv), None, P(sm), P(si),  # noqa: E731
                                   0.1, 1e-5, 1, 1, None, 0, 1, P(ws), ws.numel(), st)
fn = lambda: lib.rtsds_bn_bwd(P(dy), P(x), None, P(dx), None, P(dg), P(db), rows, c, P(g), P(b), P(sm), P(si),  # noqa: E731
                              1, 1, 0, 1, P(ws), ws.numel(), st)
if os.environ.get("BN_Y"):  # residual BatchNorm + ReLU: mask from y, dres = dy * relu'(y) as well
    yy, dres = torch.randn(rows, c, device=dev).to(torch.bfloat16), torch.empty_like(x)
    fn = lambda: lib.rtsds_bn_bwd(P(dy), P(x), P(yy), P(dx), P(dres), P(dg), P(db), rows, c, P(g), P(b), P(sm),  # noqa: E731
                                  P(si), 1, 1, 0, 1, P(ws), ws.numel(), st)
if os.environ.get("BN_FWD"):
    fn = fwd  # noqa: F811
for _ in range(3):
    fn()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(iters):
    fn()
e1.record()
torch.cuda.synchronize()
t = e0.elapsed_time(e1) / iters * 1e3
print(f"bn_bwd rows={rows} c={c}: {t:7.1f} us  ({5 * rows * c * 2 / t / 1e6:.2f} TB/s over 2R+2R+1W)")
