"""Checkpoint interchange on the HIP path (reference train.py:310-314
saves ``generator.state_dict()`` / ``discriminator.state_dict()``):

* model state_dicts move rtsds -> oracle (reference layout) and back with equal outputs;
* optimizer state (torch.optim format) saved mid-training and restored into a fresh
  optimizer resumes bit-identically; the same state drives torch.optim.Adam / SGD on the
  oracle model to the same update (interchange with the reference's optimizers);
* SGD (main.py:118-120) matches torch.optim.SGD, eager and hipGraph-replayed.
"""
import io

import pytest
import torch

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)

import rtsds_amd  # noqa: E402
from oracle import models as om  # noqa: E402
from oracle.weights import apply_recipe, synthetic_images, synthetic_labels  # noqa: E402
from rtsds_amd import losses, optim  # noqa: E402
from rtsds_amd import train as rtrain  # noqa: E402
from rtsds_amd.models.bisenet.build_bisenet import BiSeNet  # noqa: E402
from rtsds_amd.models.domain_shift.adversarial.model import TinyDomainDiscriminator  # noqa: E402

DEV = "cuda"


def _roundtrip(obj):
    buf = io.BytesIO()
    torch.save(obj, buf)
    buf.seek(0)
    return torch.load(buf, weights_only=True)


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).abs().max() / b.abs().max()).item()


def test_model_state_dict_interchange_both_ways():
    x = synthetic_images(2, 64, 128, seed=42)
    y = synthetic_labels(2, 64, 128, seed=43)
    # train the rtsds model one step so its weights are not the recipe's, then hand the
    # checkpoint to the reference-layout module
    net = apply_recipe(BiSeNet(19, "resnet18"), seed=1).to(DEV).train()
    opt = optim.Adam(net.parameters(), lr=1e-3)
    with rtsds_amd.precision(torch.float32):
        rtrain.seg_step(net, losses.CrossEntropyLoss(ignore_index=19), opt, x.to(DEV), y.to(DEV))
    sd = _roundtrip(net.state_dict())
    ref = om.BiSeNet(19, "resnet18")
    ref.load_state_dict(sd)
    ref.eval()
    net.eval()
    with torch.no_grad():
        want = ref(x)
        with rtsds_amd.precision(torch.float32):
            got = net(x.to(DEV))
    assert _rel(got, want) < 1e-3
    # and the other way: a reference-layout checkpoint into a fresh rtsds model
    ref2 = apply_recipe(om.BiSeNet(19, "resnet18"), seed=9).eval()
    net2 = BiSeNet(19, "resnet18")
    net2.load_state_dict(_roundtrip(ref2.state_dict()))
    net2 = net2.to(DEV).eval()
    with torch.no_grad():
        want = ref2(x)
        with rtsds_amd.precision(torch.float32):
            got = net2(x.to(DEV))
    assert _rel(got, want) < 1e-3
    d = apply_recipe(TinyDomainDiscriminator(19), seed=2)
    od = om.TinyDomainDiscriminator(19)
    od.load_state_dict(_roundtrip(d.state_dict()))
    for (k, a), (_, b) in zip(d.state_dict().items(), od.state_dict().items()):
        assert torch.equal(a, b), k


def _run(net, opt, x, y, steps):
    ce = losses.CrossEntropyLoss(ignore_index=19)
    for _ in range(steps):
        rtrain.seg_step(net, ce, opt, x, y)
    torch.cuda.synchronize()


@pytest.mark.parametrize("kind", ["adam", "sgd"])
def test_optimizer_resume_bit_identical(kind):
    """3 steps straight == 2 steps, save (model + optimizer), restore into fresh objects,
    1 step -- bit-identical parameters and optimizer state."""
    x = synthetic_images(2, 64, 128, seed=42).to(DEV)
    y = synthetic_labels(2, 64, 128, seed=43).to(DEV)
    make = ((lambda p: optim.Adam(p, lr=1e-3, weight_decay=1e-4)) if kind == "adam"
            else (lambda p: optim.SGD(p, lr=1e-2, momentum=0.9)))
    with rtsds_amd.precision(torch.bfloat16):
        a = apply_recipe(BiSeNet(19, "resnet18"), seed=1).to(DEV).train()
        oa = make(a.parameters())
        _run(a, oa, x, y, 3)
        b = apply_recipe(BiSeNet(19, "resnet18"), seed=1).to(DEV).train()
        ob = make(b.parameters())
        _run(b, ob, x, y, 2)
        ck = _roundtrip({"model": b.state_dict(), "opt": ob.state_dict()})
        c = BiSeNet(19, "resnet18")
        c.load_state_dict(ck["model"])
        c = c.to(DEV).train()
        oc = make(c.parameters())
        oc.load_state_dict(ck["opt"])
        _run(c, oc, x, y, 1)
    for (k, p), (_, q) in zip(a.state_dict().items(), c.state_dict().items()):
        assert torch.equal(p, q), k
    sa, sc = oa.state_dict(), oc.state_dict()
    for i in sa["state"]:
        for key, v in sa["state"][i].items():
            assert torch.equal(v, sc["state"][i][key]), (i, key)


@pytest.mark.parametrize("kind", ["adam", "sgd"])
def test_optimizer_state_interchanges_with_torch(kind):
    """An rtsds optimizer's state_dict loads into torch.optim (the reference's optimizer) on
    the oracle model, and one more step from identical gradients gives the same parameters
    (fp32; 1e-6 relative, the kernels' fma order) -- and torch's state loads back."""
    torch.manual_seed(0)
    shapes = [(64, 19, 4, 4), (64,), (1, 64, 4, 4), (1,)]
    params = [torch.nn.Parameter(torch.randn(s)) for s in shapes]
    dparams = [torch.nn.Parameter(p.detach().clone().to(DEV)) for p in params]
    if kind == "adam":
        ours, theirs = optim.Adam(dparams, lr=1e-3, weight_decay=1e-4), torch.optim.Adam(params, lr=1e-3, weight_decay=1e-4)
    else:
        ours = optim.SGD(dparams, lr=1e-2, momentum=0.9, weight_decay=1e-4)
        theirs = torch.optim.SGD(params, lr=1e-2, momentum=0.9, weight_decay=1e-4)
    gen = torch.Generator().manual_seed(3)
    for it in range(3):
        grads = [torch.randn(s, generator=gen) for s in shapes]
        ours.zero_grad()
        for p, g in zip(dparams, grads):
            p.grad.copy_(g.to(DEV))
            p._rt_arena[0].touched[p._rt_arena[1]] = True
        ours.step()
        if it == 1:  # hand the state over after two steps
            with torch.no_grad():
                for p, q in zip(params, dparams):
                    p.copy_(q.cpu())
            theirs.load_state_dict(_roundtrip(ours.state_dict()))
        if it == 2:
            for p, g in zip(params, grads):
                p.grad = g.clone()
            theirs.step()
    torch.cuda.synchronize()
    for p, q in zip(params, dparams):
        assert torch.allclose(q.detach().cpu(), p.detach(), rtol=1e-6, atol=1e-7)
    back = optim.Adam if kind == "adam" else optim.SGD
    fresh = [torch.nn.Parameter(p.detach().clone().to(DEV)) for p in params]
    o2 = back(fresh, lr=1e-3) if kind == "adam" else back(fresh, lr=1e-2, momentum=0.9, weight_decay=1e-4)
    o2.load_state_dict(_roundtrip(theirs.state_dict()))
    st = o2.state_dict()["state"]
    for i, p in enumerate(params):
        ref = theirs.state[p]
        key = "exp_avg" if kind == "adam" else "momentum_buffer"
        assert torch.allclose(st[i][key].cpu(), ref[key], rtol=0, atol=0), i


def test_sgd_matches_torch_and_graph_replay():
    """rtsds SGD (momentum 0.9, weight decay, nesterov off / on) vs torch.optim.SGD over 4
    steps; and a hipGraph replay of a seg iteration with SGD equals the eager iteration."""
    from rtsds_amd.runtime import GraphedStep
    for nesterov in (False, True):
        torch.manual_seed(1)
        shapes = [(32, 16, 3, 3), (32,)]
        params = [torch.nn.Parameter(torch.randn(s)) for s in shapes]
        dparams = [torch.nn.Parameter(p.detach().clone().to(DEV)) for p in params]
        ours = optim.SGD(dparams, lr=1e-2, momentum=0.9, weight_decay=1e-3, nesterov=nesterov)
        theirs = torch.optim.SGD(params, lr=1e-2, momentum=0.9, weight_decay=1e-3, nesterov=nesterov)
        gen = torch.Generator().manual_seed(4)
        for _ in range(4):
            grads = [torch.randn(s, generator=gen) for s in shapes]
            ours.zero_grad()
            for p, g in zip(dparams, grads):
                p.grad.copy_(g.to(DEV))
                p._rt_arena[0].touched[p._rt_arena[1]] = True
            ours.step()
            for p, g in zip(params, grads):
                p.grad = g.clone()
            theirs.step()
        torch.cuda.synchronize()
        for p, q in zip(params, dparams):
            assert torch.allclose(q.detach().cpu(), p.detach(), rtol=1e-6, atol=1e-7)
    x = synthetic_images(2, 64, 128, seed=42).to(DEV)
    y = synthetic_labels(2, 64, 128, seed=43).to(DEV)
    ce = losses.CrossEntropyLoss(ignore_index=19)
    states = []
    with rtsds_amd.precision(torch.bfloat16):
        for graphed in (False, True):
            net = apply_recipe(BiSeNet(19, "resnet18"), seed=1).to(DEV).train()
            opt = optim.SGD(net.parameters(), lr=1e-2, momentum=0.9)

            def core():
                return rtrain.seg_step(net, ce, opt, x, y)
            core()
            run = GraphedStep(core, [opt], warmup=0) if graphed else core
            for i in range(3):
                opt.param_groups[0]["lr"] = 1e-2 * (1 - i / 10)
                run()
            torch.cuda.synchronize()
            states.append({k: v.detach().float().cpu() for k, v in net.state_dict().items()})
    for k in states[0]:
        assert torch.equal(states[0][k], states[1][k]), k
