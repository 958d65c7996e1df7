"""Determinism probe: the same bf16 conv forward launched 3x on identical inputs must be
bit-identical.  Prints the mismatch count per geometry."""
import sys, math
import torch
sys.path.insert(0, ".")
import rtsds_amd
from rtsds_amd import functional as F
from rtsds_amd.nn import _shadow
CL = torch.channels_last
geos = [
    (8, 19, 512, 1024, 64, 4, 4, 2, 2, 1, 1, 1, 1),
    (8, 32, 512, 1024, 64, 4, 4, 2, 2, 1, 1, 1, 1),
    (8, 64, 256, 512, 64, 4, 4, 2, 2, 1, 1, 1, 1),
    (1, 19, 512, 1024, 64, 4, 4, 2, 2, 1, 1, 1, 1),
    (8, 32, 256, 512, 64, 3, 3, 1, 1, 1, 1, 1, 1),
    (8, 32, 512, 1024, 64, 4, 4, 2, 2, 1, 1, 1, 1, "bias"),
]
for g in geos:
    n, c, h, w, k, kh, kw, sh, sw, ph, pw, dh, dw = g[:13]
    gen = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(n, c, h, w, device="cuda", generator=gen).to(torch.bfloat16).contiguous(memory_format=CL)
    wt = (torch.randn(k, c, kh, kw, device="cuda", generator=gen) / math.sqrt(c * kh * kw)).contiguous(memory_format=CL)
    b = torch.randn(k, device="cuda", generator=gen) if len(g) > 13 else None
    with rtsds_amd.precision(torch.bfloat16), torch.no_grad():
        ys = [F.conv2d(x, wt, b, _shadow(wt, torch.bfloat16), (sh, sw), (ph, pw), (dh, dw), 0) for _ in range(3)]
    torch.cuda.synchronize()
    d = [int((ys[0] != y).sum()) for y in ys[1:]]
    print(g, "mismatches vs first:", d, flush=True)

# hconv (halo direct conv) geometries: FFM 1024 -> 19 at bs8 64x128, layer3 256 -> 256 at 32x64
for g in [(8, 1024, 64, 128, 19, 3, 3, 1, 1, 1, 1, 1, 1), (8, 256, 32, 64, 256, 3, 3, 1, 1, 1, 1, 1, 1)]:
    n, c, h, w, k, kh, kw, sh, sw, ph, pw, dh, dw = g
    gen = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(n, c, h, w, device="cuda", generator=gen).to(torch.bfloat16).contiguous(memory_format=CL)
    wt = (torch.randn(k, c, kh, kw, device="cuda", generator=gen) / math.sqrt(c * kh * kw)).contiguous(memory_format=CL)
    with rtsds_amd.precision(torch.bfloat16), torch.no_grad():
        ys = [F.conv2d(x, wt, None, _shadow(wt, torch.bfloat16), (sh, sw), (ph, pw), (dh, dw), 0) for _ in range(5)]
    torch.cuda.synchronize()
    print(g, "mismatches vs first:", [int((ys[0] != y).sum()) for y in ys[1:]], flush=True)
