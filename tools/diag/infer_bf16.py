"""Diagnostic: where the bf16 eval forward departs from fp32 mode (bench inference workload,
8 x 3 x 512 x 1024).  Prints the whole-network relative Frobenius error / argmax agreement of
(a) the graphed fast path, (b) the unfused no-grad path, (c) the autograd eval path, each bf16 vs
its fp32 counterpart; (d) per-module teacher-forced errors (each module fed the SAME bf16-exact
input in both precisions); (e) controls: fp32 on the bf16-rounded input, and fp32 with every
module output rounded to bf16."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import rtsds_amd  # noqa: E402
from oracle import models as om  # noqa: E402
from oracle.weights import recipe_state_dict, synthetic_images  # noqa: E402
from rtsds_amd.models.bisenet.build_bisenet import BiSeNet  # noqa: E402
from rtsds_amd.runtime import GraphedForward  # noqa: E402

DEV = "cuda"
NC = 19


def state(nstat):
    ref = om.BiSeNet(NC, "resnet18")
    sd = ref.state_dict()
    ref.load_state_dict(recipe_state_dict({k: tuple(v.shape) for k, v in sd.items()}, 1))
    bns = [m for m in ref.modules() if isinstance(m, torch.nn.BatchNorm2d)]
    for m in bns:
        m.momentum = 1.0
    torch.set_num_threads(16)
    with torch.no_grad():
        ref.train()(synthetic_images(nstat, 512, 1024, seed=50))
    return {k: v.clone() for k, v in ref.state_dict().items()}


def cmp(a, b):
    return ((a - b).norm() / b.norm()).item(), (a.argmax(1) == b.argmax(1)).float().mean().item()


def main():
    nstat = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    sd = state(nstat)
    net = BiSeNet(NC, "resnet18")
    net.load_state_dict(sd)
    net = net.to(DEV).eval()
    g = torch.Generator().manual_seed(42)
    x = torch.randint(0, 256, (8, 3, 512, 1024), generator=g).float()
    x = ((x - torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)) / torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)).to(DEV)
    out = {}

    def graphed(dt, xx):
        with rtsds_amd.precision(dt), torch.no_grad():
            f = GraphedForward(net, xx)
            return f(xx).float().clone()

    def nograd(dt, xx, fused=True):
        BiSeNet.inference_fusions = fused
        try:
            with rtsds_amd.precision(dt), torch.no_grad():
                return net(xx).float().clone()
        finally:
            BiSeNet.inference_fusions = True

    def general(dt, xx):
        with rtsds_amd.precision(dt):
            return net(xx).detach().float().clone()
    r32 = graphed(torch.float32, x)
    print(f"stats from {nstat} images")
    print("graphed fast bf16 vs fp32       fro %.4f argmax %.4f" % cmp(graphed(torch.bfloat16, x), r32))
    print("control: fp32 on bf16 input     fro %.4f argmax %.4f" % cmp(graphed(torch.float32, x.bfloat16().float()), r32))
    u32 = nograd(torch.float32, x, False)
    print("unfused fp32 vs fast fp32       fro %.2e argmax %.4f" % cmp(u32, r32))
    print("unfused bf16 vs unfused fp32    fro %.4f argmax %.4f" % cmp(nograd(torch.bfloat16, x, False), u32))
    g32 = general(torch.float32, x[:4])
    print("autograd-eval bf16 vs fp32 (bs4) fro %.4f argmax %.4f" % cmp(general(torch.bfloat16, x[:4]), g32))
    # (d) teacher-forced modules
    cp = net.context_path
    mods = [(f"saptial_path.convblock{i}", getattr(net.saptial_path, f"convblock{i}")) for i in (1, 2, 3)]
    mods += [(f"context_path.layer{li}.{bi}", blk) for li in (1, 2, 3, 4)
             for bi, blk in enumerate(getattr(cp, f"layer{li}"))]
    rec = {}
    hooks = [m.register_forward_pre_hook(lambda mod, args, n=n: rec.__setitem__(n, args[0].detach().float().clone()))
             for n, m in mods]
    nograd(torch.float32, x[:2], False)
    for h in hooks:
        h.remove()
    md = dict(mods)
    for n in rec:
        inp = rec[n].bfloat16()
        with torch.no_grad():
            with rtsds_amd.precision(torch.bfloat16):
                a = md[n](inp).float()
            with rtsds_amd.precision(torch.float32):
                b = md[n](inp.float()).float()
        print(f"  teacher-forced {n:28s} fro {cmp(a, b)[0]:.4f}")
    # (e) every module output rounded to bf16 in fp32 mode
    leafs = [m for n, m in net.named_modules() if n and len(list(m.children())) == 0]

    def rnd(mod, args, o):
        return o.bfloat16().float() if isinstance(o, torch.Tensor) and o.dtype == torch.float32 else o
    hooks = [m.register_forward_hook(rnd) for _, m in mods]
    print("control: fp32, module outputs rounded   fro %.4f argmax %.4f" % cmp(nograd(torch.float32, x, False), u32))
    for h in hooks:
        h.remove()
    # (f) the ARM attention (GAP -> 1x1 conv -> BN -> sigmoid on [N, C, 1, 1]) in fp32 mode from
    # the fp32 pooled features, the attention rounded to bf16 afterwards
    from rtsds_amd.models.bisenet.build_bisenet import AttentionRefinementModule as ARM
    orig = ARM.attention

    def att32(self, input, pooled=None):
        with rtsds_amd.precision(torch.float32):
            p32 = None if pooled is None else pooled.float()
            a = orig(self, input.float(), p32)
        return a.to(input.dtype)
    ARM.attention = att32
    try:
        print("fp32 ARM attention: bf16 vs fp32  fro %.4f argmax %.4f" % cmp(nograd(torch.bfloat16, x, False), u32))
    finally:
        ARM.attention = orig
    # ARM attention sensitivity: pooled-feature statistics of the ARM BatchNorms
    for nm in ("attention_refinement_module1", "attention_refinement_module2"):
        bn = getattr(net, nm).bn
        gain = (bn.weight.abs() / (bn.running_var + bn.eps).sqrt())
        print(f"{nm}.bn gain |gamma|/sqrt(var+eps): median {gain.median().item():.1f} max {gain.max().item():.1f}")


if __name__ == "__main__":
    main()
