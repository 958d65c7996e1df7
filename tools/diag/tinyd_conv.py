"""Diagnose the TinyD conv1 geometry (8x19x512x1024 -> 64, k4 s2 p1) in bf16: forward checked
before the backward, operands re-checked after it (out-of-bounds writes), 4 repetitions."""
import sys
import torch
sys.path.insert(0, ".")
from tests.test_configs_gpu import _fwd_ref, _dgrad_ref, _wgrad_ref, _check, CL, DEV
import rtsds_amd
from rtsds_amd import functional as F
from rtsds_amd.nn import _shadow
import math

g = (8, 19, 512, 1024, 64, 4, 4, 2, 2, 1, 1, 1, 1)
n, c, h, w, k, kh, kw, sh, sw, ph, pw, dh, dw = g
for rep in range(4):
    gen = torch.Generator(device=DEV).manual_seed(1000 + rep)
    x = torch.randn(n, c, h, w, device=DEV, generator=gen).to(torch.bfloat16).contiguous(memory_format=CL)
    wt = (torch.randn(k, c, kh, kw, device=DEV, generator=gen) / math.sqrt(c * kh * kw)).to(torch.bfloat16).float().contiguous(memory_format=CL)
    wp = torch.nn.Parameter(wt.clone())
    xd = x.clone().requires_grad_(True)
    with rtsds_amd.precision(torch.bfloat16):
        y = F.conv2d(xd, wp, None, _shadow(wp, torch.bfloat16), (sh, sw), (ph, pw), (dh, dw), 0)
        torch.cuda.synchronize()
        ho_n, wo_n = y.shape[2], y.shape[3]
        P = 4096
        pix = tuple(torch.randint(0, m, (P,), device=DEV, generator=gen) for m in (n, ho_n, wo_n))
        yref = _fwd_ref(x, wt, None, pix, g)
        got = y[pix[0], :, pix[1], pix[2]]
        err = (got.double() - yref).abs()
        bad = err > 8e-3 * yref.abs() + 2e-3 * yref.abs().max()
        print(rep, "fwd before bwd: bad", int(bad.sum()), "max err", float(err.max()), flush=True)
        if bad.any():
            idx = bad.nonzero()[:10]
            for p_, ch in idx.tolist():
                print("   n", int(pix[0][p_]), "ho", int(pix[1][p_]), "wo", int(pix[2][p_]), "k", ch,
                      float(got[p_, ch]), float(yref[p_, ch]))
        y0, x0 = y.detach().clone(), xd.detach().clone()
        dy = torch.randn(y.shape, device=DEV, generator=gen).to(torch.bfloat16).contiguous(memory_format=CL)
        y.backward(dy)
        torch.cuda.synchronize()
        print(rep, "y intact", torch.equal(y0, y.detach()), "x intact", torch.equal(x0, xd.detach()), flush=True)
        # full forward recompute vs first
        y2 = F.conv2d(x.clone(), wp.detach(), None, _shadow(wp, torch.bfloat16), (sh, sw), (ph, pw), (dh, dw), 0)
        torch.cuda.synchronize()
        print(rep, "fwd deterministic", torch.equal(y2, y0), int((y2 != y0).sum()), flush=True)
