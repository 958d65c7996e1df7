"""Graph capture of the overlapped DA iteration under variants (diagnosis of a capture_end
fault): argv[1] in {base, nobranch, norecord}."""
import os
import sys
import faulthandler
faulthandler.enable()
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

import rtsds_amd
from rtsds_amd import losses, optim
from rtsds_amd import train as rtrain
from rtsds_amd.models.bisenet.build_bisenet import BiSeNet
from rtsds_amd.models.domain_shift.adversarial.model import TinyDomainDiscriminator
from rtsds_amd.runtime import GraphedStep

v = sys.argv[1]
dev = "cuda"
g = torch.Generator().manual_seed(17)
x = torch.randn(2, 3, 128, 256, generator=g).to(dev)
xt = torch.randn(2, 3, 128, 256, generator=g).to(dev)
y = torch.randint(0, 20, (2, 128, 256), generator=g).to(dev)
ce, bce = losses.CrossEntropyLoss(ignore_index=19), losses.BCEWithLogitsLoss()
if v == "norecord":
    torch.Tensor.record_stream = lambda self, s: None
with rtsds_amd.precision(torch.bfloat16):
    net = BiSeNet(19, "resnet18").to(dev).train()
    if v == "nobranch":
        net.branch_parallel = False
    disc = TinyDomainDiscriminator(19).to(dev).train()
    opt = optim.Adam(net.parameters(), lr=1e-3)
    dopt = optim.Adam(disc.parameters(), lr=1e-3)
    core = lambda: rtrain.da_step(net, disc, opt, dopt, ce, bce, x, y, xt, 0.1, 2)  # noqa: E731
    step = GraphedStep(core, [opt, dopt], warmup=1)
    print(v, [float(t) for t in step()], flush=True)
