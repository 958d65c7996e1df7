"""Where does DeepLabV2 bf16 diverge from fp32 mode?  Per-block relative error (forward hooks)
at 97x129 batch 1 and 1024x512 batch 1; plus the oracle control (input rounded to bf16)."""
import sys
import torch
sys.path.insert(0, ".")
import rtsds_amd
from oracle import models as om
from oracle.weights import synthetic_images
from tests.test_configs_gpu import _load
from rtsds_amd.models.deeplabv2.deeplabv2 import get_deeplab_v2

for (h, w) in ((97, 129), (512, 1024)):
    x = synthetic_images(1, h, w, seed=44)
    outs = {}
    for dt in (torch.float32, torch.bfloat16):
        net = _load(get_deeplab_v2(19, pretrain=False), 3).cuda().train()
        rec = []
        for name, m in net.named_modules():
            if name.count(".") == 1 and name.startswith("layer") or name in ("layer6",):
                m.register_forward_hook(lambda mod, inp, out, name=name: rec.append((name, out.detach().float().clone())))
        with torch.no_grad(), rtsds_amd.precision(dt):
            o, _, _ = net(x.cuda())
        outs[dt] = (o.float(), rec)
    a, b = outs[torch.bfloat16], outs[torch.float32]
    for (n1, t1), (n2, t2) in zip(a[1], b[1]):
        print(h, w, n1, "rel fro", float((t1 - t2).norm() / t2.norm()), "max", float(t2.abs().max()), flush=True)
    print(h, w, "out rel fro", float((a[0] - b[0]).norm() / b[0].norm()))
    if h < 200:
        ref = _load(om.ResNetMulti(), 3).train()
        with torch.no_grad():
            r1, _, _ = ref(x)
            r2, _, _ = ref(x.bfloat16().float())
        print("oracle control fro", float((r1 - r2).norm() / r1.norm()), "ours fp32 vs oracle",
              float((b[0].cpu() - r1).norm() / r1.norm()))
