"""Reproduce test_graphed_step_with_collectives[True] step by step with prints."""
import socket, sys, traceback
import torch
import torch.distributed as dist
sys.path.insert(0, ".")
import rtsds_amd
from rtsds_amd import functional as rf, losses as rl, optim, train as rtrain, runtime
from rtsds_amd.runtime import GraphedStep
from rtsds_amd.models.bisenet.build_bisenet import BiSeNet
from rtsds_amd.models.domain_shift.adversarial.model import TinyDomainDiscriminator
DEV = "cuda"
with socket.socket() as s:
    s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]
dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
for mod in (rf, optim, rl, rtrain):
    mod.dp_world = lambda: 2
g = torch.Generator().manual_seed(11)
x = torch.randn(2, 3, 64, 128, generator=g).to(DEV)
xt = torch.randn(2, 3, 64, 128, generator=g).to(DEV)
y = torch.randint(0, 20, (2, 64, 128), generator=g).to(DEV)
ce, bce = rl.CrossEntropyLoss(ignore_index=19), rl.BCEWithLogitsLoss()
states = []
try:
    with rtsds_amd.precision(torch.bfloat16):
        for overlap, graphed in ((False, False), (True, False), (True, True)):
            print("variant", overlap, graphed, flush=True)
            optim.set_overlap_allreduce(overlap)
            torch.manual_seed(3)
            net = BiSeNet(19, "resnet18").to(DEV).train()
            disc = TinyDomainDiscriminator(19).to(DEV).train()
            opt = optim.Adam(net.parameters(), lr=1e-3)
            dopt = optim.Adam(disc.parameters(), lr=1e-3, weight_decay=1e-4)
            def core():
                return rtrain.da_step(net, disc, opt, dopt, ce, bce, x, y, xt, 0.1, 100)[0]
            run = core
            for i in range(4):
                if graphed and i == 1:
                    run = GraphedStep(core, [opt, dopt], warmup=0)
                    print("segments", len(run.segments), flush=True)
                run()
                torch.cuda.synchronize()
                print(" iter", i, "ok", flush=True)
            states.append({k: v.detach().float().cpu().clone() for k, v in
                           list(net.state_dict().items()) + list(disc.state_dict().items())})
    for st in states[1:]:
        bad = [k for k in states[0] if not torch.equal(states[0][k], st[k])]
        print("mismatching keys:", len(bad), bad[:5], flush=True)
except Exception:
    traceback.print_exc()
    sys.stdout.flush()
print("destroying", flush=True)
dist.destroy_process_group()
print("done", flush=True)
