"""Fused upsample + CE at small factors vs torch fp64, per head count (diagnostic)."""
import os
import sys

import torch
import torch.nn.functional as TF

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from rtsds_amd import functional as F  # noqa: E402

for sf, k, hl, wl in ((2, 1, 8, 16), (2, 2, 8, 16), (2, 3, 8, 16), (4, 3, 8, 16), (3, 3, 8, 16), (2, 3, 16, 32), (2, 1, 4, 4)):
    g = torch.Generator().manual_seed(21)
    heads = [torch.randn(2, 19, hl, wl, generator=g, dtype=torch.float64) * 2 for _ in range(k)]
    hd = [h.float().cuda() for h in heads]
    geo = F.upsample_geometry(hd[0], scale_factor=sf)
    H, W = geo[0], geo[1]
    t = torch.randint(0, 20, (2, H, W), generator=g)
    t[t == 19] = 255
    ref = [float(TF.cross_entropy(TF.interpolate(h, scale_factor=sf, mode="bilinear", align_corners=False), t,
                                  ignore_index=255)) for h in heads]
    ok = F.upsample_cross_entropy_supported(hd, geo, 255)
    got = [float(F.upsample_cross_entropy([h], t.cuda(), geo, 255)) for h in hd] if ok else None
    tot = float(F.upsample_cross_entropy(hd, t.cuda(), geo, 255)) if ok else None
    print(f"x{sf} heads {k} {hl}x{wl}: supported {ok}  ref {sum(ref):.5f} fused {tot}  per-head-alone {got} ref {ref}", flush=True)
