"""Diagnostic: spatial-path gradient precision per stage vs fp64 CPU."""
import sys, torch
sys.path.insert(0, '.')
import rtsds_amd
from oracle import models as om
from oracle.weights import recipe_state_dict, synthetic_images
from rtsds_amd.models.bisenet.build_bisenet import Spatial_path
from rtsds_amd.nn import to_input

x = synthetic_images(2, 128, 256, seed=42)
def load(m):
    sd = m.state_dict(); m.load_state_dict(recipe_state_dict({k: tuple(v.shape) for k, v in sd.items()}, 1)); return m
g = torch.Generator().manual_seed(0)
gy = torch.randn(2, 256, 16, 32, generator=g, dtype=torch.float64)
fro = lambda a, b: ((a.double().cpu() - b.double().cpu()).norm() / b.double().norm()).item()
res = {}
for dt in (torch.float64, torch.float32):
    m = load(om.Spatial_path()).to(dt).train()
    acts = {}
    h1 = m.convblock1.conv1(x.to(dt)); h1.retain_grad()
    a1 = m.convblock1(x.to(dt)); 
    out = m(x.to(dt))
    out.backward(gy.to(dt))
    res[dt] = {k: p.grad for k, p in m.named_parameters()}
m = load(Spatial_path()).cuda().train()
with rtsds_amd.precision(torch.float32):
    out = m(to_input(x.cuda()))
    out.backward(gy.float().cuda().contiguous(memory_format=torch.channels_last))
for k, p in m.named_parameters():
    print(f"{k:40s} ours {fro(p.grad, res[torch.float64][k]):.2e}  cpu32 {fro(res[torch.float32][k], res[torch.float64][k]):.2e}")
