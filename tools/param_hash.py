"""Bit-identity check across library builds: a few seeded BiSeNet bf16 train steps (eager, then
hipGraph replays), printing the losses and a SHA-256 of every parameter, buffer and optimizer
moment.  Run once per build (RTSDS_LIB=...) and compare the lines."""
import hashlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import rtsds_amd  # noqa: E402
from rtsds_amd import losses, optim  # noqa: E402
from rtsds_amd import train as rtrain  # noqa: E402
from rtsds_amd.models.bisenet.build_bisenet import BiSeNet  # noqa: E402
from rtsds_amd.runtime import GraphedStep  # noqa: E402

dev = torch.device("cuda")
g = torch.Generator().manual_seed(21)
x = torch.randn(8, 3, 256, 512, generator=g).to(dev)
y = torch.randint(0, 20, (8, 256, 512), generator=g).to(dev)
ce = losses.CrossEntropyLoss(ignore_index=19)
with rtsds_amd.precision(torch.bfloat16):
    for graphed in (False, True):
        torch.manual_seed(9)
        net = BiSeNet(19, "resnet18").to(dev).train()
        opt = optim.Adam(net.parameters(), lr=1e-3)
        core = lambda: rtrain.seg_step(net, ce, opt, x, y)  # noqa: E731
        step = GraphedStep(core, [opt], warmup=1) if graphed else core
        ls = [[float(v) for v in step()] for _ in range(4)]
        torch.cuda.synchronize()
        h = hashlib.sha256()
        for k, v in net.state_dict().items():
            h.update(v.detach().float().cpu().numpy().tobytes())
        for a in opt.arenas():
            h.update(a.m.cpu().numpy().tobytes())
        print("graphed" if graphed else "eager", ls, h.hexdigest(), flush=True)
