"""Data-parallel semantics on one GPU (two ranks, gloo): a sharded seg step must equal the
reference's DataParallel step on the gathered batch -- per-replica BatchNorm statistics, but
ONE cross-entropy mean over every rank's non-ignored pixels (reference
utils.forModel -> nn.DataParallel, train.py:86-92).  The two shards get very different
ignore fractions, so a mean of per-rank means would fail this test.  Both generators: BiSeNet
(one backward bucket cut) and a short DeepLabV2 (ResNetMulti with [1, 1, 3, 1] Bottlenecks: the
same three grad_cut points as the full [3, 4, 23, 3] net, so G's gradient is all-reduced in four
buckets while the backward proceeds, runtime.grad_cut / train.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data():
    from oracle.weights import synthetic_images, synthetic_labels
    x = synthetic_images(4, 64, 128, seed=42)
    y = synthetic_labels(4, 64, 128, seed=43)
    y[:2][torch.rand(y[:2].shape, generator=torch.Generator().manual_seed(5)) < 0.5] = 19
    return x, y


KINDS = ("bisenet", "deeplab")


def _model(kind="bisenet"):
    from oracle.weights import recipe_state_dict
    if kind == "bisenet":
        from rtsds_amd.models.bisenet.build_bisenet import BiSeNet
        net = BiSeNet(19, "resnet18")
    else:
        from rtsds_amd.models.deeplabv2.deeplabv2 import Bottleneck, ResNetMulti
        net = ResNetMulti(Bottleneck, [1, 1, 3, 1], 19)
    sd = net.state_dict()
    net.load_state_dict(recipe_state_dict({k: tuple(v.shape) for k, v in sd.items()}, 1))
    return net.to(DEV).train()


def _worker(rank, world, port, out, kind):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as dist
    import rtsds_amd
    from rtsds_amd import losses, optim
    from rtsds_amd.train import seg_step
    dist.init_process_group("gloo")
    starts = []
    orig = optim.allreduce_start

    def spy(bufs, wires=None):  # one call per gradient bucket
        starts.append(len(bufs))
        return orig(bufs, wires)
    optim.allreduce_start = spy
    try:
        x, y = _data()
        xs, ys = x[2 * rank:2 * rank + 2].to(DEV), y[2 * rank:2 * rank + 2].to(DEV)
        with rtsds_amd.precision(torch.float32):
            net = _model(kind)
            opt = optim.Adam(net.parameters(), lr=1e-4)
            loss, corr = seg_step(net, losses.CrossEntropyLoss(ignore_index=19), opt, xs, ys)
            t = torch.stack([loss.double(), corr[0].double()])
            dist.all_reduce(t)
        if rank == 0:
            torch.save({"loss": float(t[0]), "correct": int(t[1]), "buckets": len(starts),
                        "params": {k: v.detach().cpu() for k, v in net.named_parameters()}}, out)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind", KINDS)
def test_two_rank_seg_step_equals_gathered_batch(tmp_path, kind):
    out = str(tmp_path / "rank0.pt")
    ctx = mp.get_context("spawn")
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, out, kind)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    got = torch.load(out, weights_only=True)
    # the phased backward: a bucket per cut plus the rest (BiSeNet 1 cut, DeepLab 3)
    assert got["buckets"] >= (2 if kind == "bisenet" else 4), got["buckets"]

    # single device, DataParallel semantics: each replica's forward on its own half (its own
    # BatchNorm statistics), the losses (three heads / one) over the gathered outputs
    import rtsds_amd
    from rtsds_amd import functional as F
    from rtsds_amd import optim
    x, y = _data()
    with rtsds_amd.precision(torch.float32):
        net = _model(kind)
        opt = optim.Adam(net.parameters(), lr=1e-4)
        opt.zero_grad()
        halves = [net.forward_lowres(x[i:i + 2].to(DEV)) for i in (0, 2)]
        heads = [torch.cat([halves[0][h][0], halves[1][h][0]]).contiguous(memory_format=torch.channels_last)
                 for h in range(len(halves[0]))]
        correct = torch.zeros(1, dtype=torch.int64, device=DEV)
        loss = F.upsample_cross_entropy(heads, y.to(DEV), halves[0][0][1], 19, correct)
        loss.backward()
        opt.step()
    lv = float(loss.detach())
    assert abs(got["loss"] - lv) <= 1e-5 * abs(lv), (got["loss"], lv)
    assert got["correct"] == int(correct)
    lr, n, bad, worst = 1e-4, 0, 0, 0.0
    for k, p in net.named_parameters():
        d = (got["params"][k] - p.detach().cpu()).abs()
        n += d.numel()
        bad += int((d > 1e-6).sum())
        worst = max(worst, float(d.max()))
    # Adam's first step moves each weight by ~lr; rounding-order differences of near-zero
    # gradients may flip a few of those moves
    assert worst <= 2.05 * lr, worst
    assert bad <= 1e-3 * n, (bad, n)


# ----------------------------------------------------------------------------- DA iteration
def _da_data():
    from oracle.weights import synthetic_images, synthetic_labels
    # unequal shards: rank 0 gets 2 source + 2 target images, rank 1 gets 3 + 3 (as the
    # reference's DataParallel scatters an odd batch; BCE and CE must use the GLOBAL counts)
    x = synthetic_images(5, 64, 128, seed=42)
    y = synthetic_labels(5, 64, 128, seed=43)
    y[:2][torch.rand(y[:2].shape, generator=torch.Generator().manual_seed(5)) < 0.5] = 19
    xt = synthetic_images(5, 64, 128, seed=46)
    return x, y, xt


SHARDS = ((0, 2), (2, 5))


def _models(kind="bisenet"):
    from oracle.weights import recipe_state_dict
    from rtsds_amd.models.domain_shift.adversarial.model import TinyDomainDiscriminator
    g = _model(kind)
    d = TinyDomainDiscriminator(19)
    sd = d.state_dict()
    d.load_state_dict(recipe_state_dict({k: tuple(v.shape) for k, v in sd.items()}, 2))
    return g, d.to(DEV).train()


def _da_worker(rank, world, port, out, kind):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as dist
    import rtsds_amd
    from rtsds_amd import losses, optim
    from rtsds_amd.train import da_step
    dist.init_process_group("gloo")
    try:
        x, y, xt = _da_data()
        lo, hi = SHARDS[rank]
        with rtsds_amd.precision(torch.float32):
            g, d = _models(kind)
            og = optim.Adam(g.parameters(), lr=1e-4)
            od = optim.Adam(d.parameters(), lr=1e-4, weight_decay=1e-4)
            res = da_step(g, d, og, od, losses.CrossEntropyLoss(ignore_index=19), losses.BCEWithLogitsLoss(),
                          x[lo:hi].to(DEV), y[lo:hi].to(DEV), xt[lo:hi].to(DEV), 0.1, 2)
            t = torch.stack([v.double().reshape(()) for v in res])
            dist.all_reduce(t)
        if rank == 0:
            torch.save({"logs": t.cpu(),
                        "g": {k: v.detach().cpu() for k, v in g.named_parameters()},
                        "d": {k: v.detach().cpu() for k, v in d.named_parameters()}}, out)
    finally:
        dist.destroy_process_group()


def _wire_worker(rank, world, port, out):
    """The same sharded DA iteration twice, with the gradient all-reduce on an fp32 wire and on
    an fp16 wire (BASELINE configs[4]: "fp16+fp32 grad all-reduce").  Saves, per rank, the local
    gradients handed to the all-reduce (recorded by wrapping optim.allreduce_start /
    allreduce_flat), the reduced gradients (Arena.reduced_grad after step()) and the updated
    parameters."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as dist
    import rtsds_amd
    from rtsds_amd import losses, optim
    from rtsds_amd.train import da_step
    dist.init_process_group("gloo")
    rec = []

    def spy(orig):
        def f(bufs, wires=None):
            rec.extend((b.data_ptr(), b.detach().clone()) for b in bufs)
            return orig(bufs, wires)
        return f
    optim.allreduce_start = spy(optim.allreduce_start)
    optim.allreduce_flat = spy(optim.allreduce_flat)

    def flat(opt, local):
        parts = []
        for a in opt.arenas():
            if not local:  # the summed gradients the update applied (the wire copy for fp16)
                parts.append(a.reduced_grad().cpu())
                continue
            loc, base = torch.zeros_like(a.gflat), a.gflat.data_ptr()
            for ptr, v in rec:
                off = (ptr - base) // 4
                if 0 <= off < a.total:
                    loc[off:off + v.numel()] = v
            parts.append(loc.cpu())
        return torch.cat(parts)
    try:
        x, y, xt = _da_data()
        lo, hi = SHARDS[rank]
        res = {}
        for wire in ("fp32", "fp16"):
            optim.set_allreduce_dtype(torch.float32 if wire == "fp32" else torch.float16)
            rec.clear()
            with rtsds_amd.precision(torch.float32):
                g, d = _models()
                og = optim.Adam(g.parameters(), lr=1e-4)
                od = optim.Adam(d.parameters(), lr=1e-4, weight_decay=1e-4)
                da_step(g, d, og, od, losses.CrossEntropyLoss(ignore_index=19), losses.BCEWithLogitsLoss(),
                        x[lo:hi].to(DEV), y[lo:hi].to(DEV), xt[lo:hi].to(DEV), 0.1, 2)
                torch.cuda.synchronize()
            res[wire] = {"local_g": flat(og, True), "local_d": flat(od, True),
                         "grad_g": flat(og, False), "grad_d": flat(od, False),
                         "g": {k: v.detach().cpu() for k, v in g.named_parameters()},
                         "d": {k: v.detach().cpu() for k, v in d.named_parameters()}}
            del g, d, og, od
        optim.set_allreduce_dtype(torch.float32)
        torch.save(res, out + f".{rank}")
    finally:
        dist.destroy_process_group()


def test_two_rank_da_step_fp16_wire_allreduce(tmp_path):
    """configs[4]'s fp16 gradient all-reduce on real gradients: the sharded DA iteration (2 ranks,
    shards of 2 and 3 images) with G's and D's flat gradients summed as float16 vs as float32.
    (a) The reduced gradients equal a host emulation of the wire from the ranks' local gradients
    bit for bit: fp32 wire l0 + l1; fp16 wire fp16(fp16(l0) + fp16(l1)) (two addends: one
    correctly rounded sum in any order), and no element overflows.  (b) The Adam updates: an
    fp16-rounded gradient keeps its sign unless it underflows, so every update stays within
    Adam's first-step bound 2.05 lr of the fp32-wire one, and >= 97 % of G's and D's elements
    move identically to 1e-6."""
    out = str(tmp_path / "wire.pt")
    ctx = mp.get_context("spawn")
    port = _port()
    procs = [ctx.Process(target=_wire_worker, args=(r, 2, port, out)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    got = [torch.load(out + f".{r}", weights_only=True) for r in range(2)]
    for wire in ("fp32", "fp16"):
        for nm in ("g", "d"):
            l0, l1 = got[0][wire]["local_" + nm], got[1][wire]["local_" + nm]
            red = got[0][wire]["grad_" + nm]
            assert torch.equal(red, got[1][wire]["grad_" + nm]), (wire, nm, "ranks differ")
            if wire == "fp32":
                want = l0 + l1
            else:
                want = (l0.half().float() + l1.half().float()).half().float()
            assert torch.isfinite(red).all(), (wire, nm)
            bad = int((red != want).sum())
            print(f"{wire} wire, {nm}: max |g| {float(red.abs().max()):.3e}, "
                  f"{bad} / {red.numel()} elements differ from the host emulation")
            assert bad == 0, (wire, nm, bad)
    r32, r16 = got[0]["fp32"], got[0]["fp16"]
    dg = (r16["grad_g"] - r32["grad_g"]).abs().max().item()
    print(f"G gradient, fp16 vs fp32 wire: max |diff| {dg:.3e}")
    lr = 1e-4
    for name in ("g", "d"):
        n = same = 0
        worst = 0.0
        for k in r32[name]:
            dlt = (r16[name][k] - r32[name][k]).abs()
            n += dlt.numel()
            same += int((dlt <= 1e-6).sum())
            worst = max(worst, float(dlt.max()))
        print(f"{name}: fp16-wire update vs fp32-wire: worst {worst:.3e}, identical {same / n:.5f}")
        assert worst <= 2.05 * lr, (name, worst)
        assert same >= 0.97 * n, (name, same, n)


def _gathered_da_step(g, d, og, od, x, y, xt, lam, it):
    """adversarial_train's iteration (train.py:174-275) under nn.DataParallel on the gathered
    batch: every module runs per replica on its shard (per-replica BatchNorm statistics), the
    outputs are gathered and each loss is one mean over the whole batch."""
    import rtsds_amd.functional as F
    from rtsds_amd import losses
    bce = losses.BCEWithLogitsLoss()
    cat = lambda ts: torch.cat(ts).contiguous(memory_format=torch.channels_last)  # noqa: E731
    og.zero_grad()
    od.zero_grad()
    for p in d.parameters():
        p.requires_grad = False
    correct = torch.zeros(1, dtype=torch.int64, device=DEV)
    parts = [g.forward_lowres(x[lo:hi]) for lo, hi in SHARDS]
    geo = parts[0][0][1]
    heads = [cat([p[h][0] for p in parts]) for h in range(len(parts[0]))]
    loss_seg = F.upsample_cross_entropy(heads, y, geo, 19, correct) / it
    loss_seg.backward()
    src = F.interpolate_geometry(heads[0].detach(), geo)
    tparts = []
    for lo, hi in SHARDS:
        (t, tg), = g.forward_lowres(xt[lo:hi], main_only=True)
        tparts.append(F.interpolate_geometry(t, tg))
    pred_t = cat([d(F.softmax(t, dim=1)) for t in tparts])
    loss_adv = lam * bce(pred_t, torch.ones(pred_t.shape, device=DEV)) / it
    loss_adv.backward()
    for p in d.parameters():
        p.requires_grad = True
    pred_s = cat([d(F.softmax(src[lo:hi], dim=1)) for lo, hi in SHARDS])
    loss_ds = bce(pred_s, torch.ones(pred_s.shape, device=DEV)) / it
    loss_ds.backward()
    pred_t2 = cat([d(F.softmax(t.detach(), dim=1)) for t in tparts])
    loss_dt = bce(pred_t2, torch.zeros(pred_t2.shape, device=DEV)) / it
    loss_dt.backward()
    og.step()
    od.step()
    return [float(v.detach()) for v in (loss_seg, loss_adv, loss_ds, loss_dt)] + [int(correct)]


@pytest.mark.parametrize("kind", KINDS)
def test_two_rank_da_step_equals_gathered_batch(tmp_path, kind):
    """A sharded adversarial_train iteration (2 ranks, UNEQUAL shards of 2 and 3 source +
    target images) equals the DataParallel iteration on the gathered batch: the four losses,
    the pixel-accuracy count, and G and D after both Adam steps (D gradients summed over
    ranks, BCE over the global element count, the frozen-D adversarial gradient into G)."""
    out = str(tmp_path / "rank0_da.pt")
    ctx = mp.get_context("spawn")
    port = _port()
    procs = [ctx.Process(target=_da_worker, args=(r, 2, port, out, kind)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    got = torch.load(out, weights_only=True)

    import rtsds_amd
    from rtsds_amd import optim
    x, y, xt = _da_data()
    with rtsds_amd.precision(torch.float32):
        g, d = _models(kind)
        og = optim.Adam(g.parameters(), lr=1e-4)
        od = optim.Adam(d.parameters(), lr=1e-4, weight_decay=1e-4)
        want = _gathered_da_step(g, d, og, od, x.to(DEV), y.to(DEV), xt.to(DEV), 0.1, 2)
    logs = got["logs"].tolist()
    for i, nm in enumerate(("loss_seg", "loss_adv", "loss_dsrc", "loss_dtgt")):
        assert abs(logs[i] - want[i]) <= 1e-5 * abs(want[i]) + 1e-9, (nm, logs[i], want[i])
    assert int(logs[4]) == want[4]
    lr = 1e-4
    for name, mod in (("g", g), ("d", d)):
        n = bad = 0
        worst = 0.0
        for k, p in mod.named_parameters():
            dlt = (got[name][k] - p.detach().cpu()).abs()
            n += dlt.numel()
            bad += int((dlt > 1e-6).sum())
            worst = max(worst, float(dlt.max()))
        assert worst <= 2.05 * lr, (name, worst)
        assert bad <= 1e-3 * n, (name, bad, n)
