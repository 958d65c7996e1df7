"""Generate golden fixtures by importing the REAL reference (build container only).

Run:  python tests/golden/make_golden.py  [--ref /root/reference]

The reference is pure Python/PyTorch; it is imported read-only from ``--ref`` with
``sys.dont_write_bytecode`` and offline stubs for its missing third-party imports:
``torchvision.models`` -> ``oracle.tv_resnet`` (restated torchvision 0.18 ResNet), and
logging-only stand-ins for fvcore / wandb / tensorboard / prettytable /
torchvision.transforms (never on the arithmetic path).  Weights come from the shared
per-key recipe (``oracle.weights``), inputs from its synthetic-image recipe.

Only data leave this script: ``tests/golden/*.npz`` (inputs are regenerated from seeds,
outputs are stored as checksums + fixed-index samples + full argmax maps) and
``tests/golden/*.json``.  Nothing here runs on the GPU box.
"""
import argparse
import json
import os
import sys
import tempfile
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from oracle import tv_resnet  # noqa: E402
from oracle.weights import apply_recipe, synthetic_images, synthetic_labels  # noqa: E402
from tests.golden.fixtures import summarize, param_summary  # noqa: E402


def install_stubs():
    tv = types.ModuleType("torchvision")
    tv.models = tv_resnet
    tr = types.ModuleType("torchvision.transforms")
    trf = types.ModuleType("torchvision.transforms.functional")
    trf.to_pil_image = lambda *a, **k: None
    tr.functional = trf
    tvio = types.ModuleType("torchvision.io")
    tvio.read_image = lambda *a, **k: None
    tvio.ImageReadMode = types.SimpleNamespace(RGB="RGB", UNCHANGED="UNCHANGED", GRAY="GRAY")
    tv.transforms, tv.io = tr, tvio
    fv = types.ModuleType("fvcore")
    fvnn = types.ModuleType("fvcore.nn")
    fvnn.FlopCountAnalysis = lambda *a, **k: None
    fvnn.flop_count_table = lambda *a, **k: ""
    fv.nn = fvnn
    tb = types.ModuleType("torch.utils.tensorboard")
    tb.SummaryWriter = object
    wb = types.ModuleType("wandb")
    pt = types.ModuleType("prettytable")

    class PrettyTable:
        def add_column(self, *a, **k):
            pass

        def __str__(self):
            return ""
    pt.PrettyTable = PrettyTable
    sys.modules.update({
        "torchvision": tv, "torchvision.models": tv_resnet, "torchvision.transforms": tr,
        "torchvision.transforms.functional": trf, "torchvision.io": tvio,
        "fvcore": fv, "fvcore.nn": fvnn, "torch.utils.tensorboard": tb, "wandb": wb,
        "prettytable": pt})


class Capture:
    """Callback-protocol object (callbacks.py:1-30) that records logged values."""

    def __init__(self):
        self.batches, self.epochs = [], []

    def on_batch_end(self, batch, logs=None):
        self.batches.append(dict(logs))

    def on_epoch_end(self, epoch, logs=None):
        self.epochs.append(dict(logs))

    def on_validation_end(self, logs=None, data=None):
        self.val = logs

    def __getattr__(self, name):
        return lambda *a, **k: None


def save(name, arrays, meta):
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **arrays)
    with open(os.path.join(HERE, name + ".json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print("wrote", name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--only", default="", help="comma-separated fixture groups (default: all)")
    args = ap.parse_args()
    only = set(filter(None, args.only.split(",")))
    sys.dont_write_bytecode = True
    install_stubs()
    sys.path.insert(0, args.ref)
    torch.manual_seed(42)
    torch.set_num_threads(8)

    from models.bisenet.build_bisenet import BiSeNet
    from models.deeplabv2.deeplabv2 import get_deeplab_v2
    from models.domain_shift.adversarial.model import DomainDiscriminator, TinyDomainDiscriminator
    import train as ref_train

    if only:
        if "inputs" in only:
            make_inputs()
        if "da2" in only:
            make_da2(ref_train, BiSeNet, TinyDomainDiscriminator)
        if "extras" in only:
            make_extras(BiSeNet, DomainDiscriminator)
        return

    keys = {}
    # ---------------- BiSeNet-R18: config 1 shape (2x3x128x256), train + eval
    g = apply_recipe(BiSeNet(19, "resnet18"), seed=1)
    keys["bisenet_r18"] = [[k, list(v.shape)] for k, v in g.state_dict().items()]
    x = synthetic_images(2, 128, 256, seed=42)
    y = synthetic_labels(2, 128, 256, seed=43)
    g.train()
    out, a1, a2 = g(x)
    ce = torch.nn.CrossEntropyLoss(ignore_index=19)
    loss = ce(out, y) + ce(a1, y) + ce(a2, y)
    loss.backward()
    arrays, meta = {}, {"loss": float(loss)}
    for nm, t in (("out", out), ("aux1", a1), ("aux2", a2)):
        summarize(arrays, meta, nm, t.detach())
    arrays["out_argmax"] = out.detach().argmax(1).to(torch.uint8).numpy()
    param_summary(arrays, meta, "grad", {k: p.grad for k, p in g.named_parameters()})
    meta["running_mean_sum"] = {k: float(v.double().sum()) for k, v in g.state_dict().items()
                                if k.endswith("running_mean")}
    g.eval()
    with torch.no_grad():
        ev = g(x)
    summarize(arrays, meta, "eval_out", ev)
    arrays["eval_argmax"] = ev.argmax(1).to(torch.uint8).numpy()
    save("bisenet_c1", arrays, meta)

    # ---------------- discriminators on softmax(random logits)
    arrays, meta = {}, {}
    z = torch.randn(2, 19, 64, 128, generator=torch.Generator().manual_seed(7))
    for nm, D in (("tiny", TinyDomainDiscriminator(19)), ("full", DomainDiscriminator(19))):
        apply_recipe(D, seed=2)
        keys["disc_" + nm] = [[k, list(v.shape)] for k, v in D.state_dict().items()]
        zi = z.clone().requires_grad_(True)
        p = D(torch.softmax(zi, 1))
        bce = torch.nn.BCEWithLogitsLoss()
        l = bce(p, torch.ones_like(p))
        l.backward()
        arrays[nm + "_pred"] = p.detach().numpy()
        meta[nm + "_loss"] = float(l)
        summarize(arrays, meta, nm + "_dz", zi.grad)
        param_summary(arrays, meta, nm + "_grad", {k: q.grad for k, q in D.named_parameters()})
    save("disc", arrays, meta)

    # ---------------- DeepLabV2 (odd size -> ceil-mode maxpool), train fwd/bwd + eval
    arrays, meta = {}, {}
    dl = apply_recipe(get_deeplab_v2(19, pretrain=False), seed=3)
    keys["deeplabv2"] = [[k, list(v.shape)] for k, v in dl.state_dict().items()]
    xd = synthetic_images(1, 97, 129, seed=44)
    yd = synthetic_labels(1, 97, 129, seed=45)
    dl.train()
    o, _, _ = dl(xd)
    l = ce(o, yd)
    l.backward()
    meta["loss"] = float(l)
    summarize(arrays, meta, "out", o.detach())
    arrays["out_argmax"] = o.detach().argmax(1).to(torch.uint8).numpy()
    param_summary(arrays, meta, "grad", {k: q.grad for k, q in dl.named_parameters()
                                         if q.grad is not None})
    save("deeplab_small", arrays, meta)

    # ---------------- one train.train epoch of one batch (train.py:24-128)
    g = apply_recipe(BiSeNet(19, "resnet18"), seed=1)
    opt = torch.optim.Adam(g.parameters(), lr=1e-4)
    cap = Capture()
    ref_train.train(epoch=0, model=g, train_loader=[(x, y.unsqueeze(1))], criterion=ce,
                    optimizer=opt, init_lr=1e-4, max_iter=4, power=0.9, lr_decay_iter=1,
                    callbacks=[cap])
    arrays, meta = {}, {"batches": cap.batches, "epochs": cap.epochs}
    param_summary(arrays, meta, "param", dict(g.named_parameters()))
    save("seg_epoch_c1", arrays, meta)

    # ---------------- adversarial_train: 1 epoch x 2 iterations (train.py:130-318)
    g = apply_recipe(BiSeNet(19, "resnet18"), seed=1)
    d = apply_recipe(TinyDomainDiscriminator(19), seed=2)
    og = torch.optim.Adam(g.parameters(), lr=1e-4)
    od = torch.optim.Adam(d.parameters(), lr=1e-4, weight_decay=1e-4)
    xt = synthetic_images(2, 128, 256, seed=46)
    cap = Capture()
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as tmp:
        os.chdir(tmp)
        try:
            ref_train.adversarial_train(
                iterations=2, epochs=1, generator=g, discriminator=d, generator_optimizer=og,
                discriminator_optimizer=od, source_dataloader=[(x, y.unsqueeze(1))],
                target_dataloader=[(xt, y.unsqueeze(1))], generator_loss=ce,
                discriminator_loss=torch.nn.BCEWithLogitsLoss(), lambda_=0.1, gen_init_lr=1e-4,
                gen_power=0.9, dis_power=0.05, dis_init_lr=1e-4, lr_decay_iter=1,
                num_classes=19, class_names=[str(i) for i in range(19)],
                val_loader=[(x, y.unsqueeze(1))], do_validation=1, callbacks=[cap])
        finally:
            os.chdir(cwd)
    arrays, meta = {}, {"batches": cap.batches, "epochs": cap.epochs,
                        "val_mIoU": float(cap.val["validation_mIoU"])}
    param_summary(arrays, meta, "gparam", dict(g.named_parameters()))
    param_summary(arrays, meta, "dparam", dict(d.named_parameters()))
    meta["g_running_mean_sum"] = {k: float(v.double().sum()) for k, v in g.state_dict().items()
                                  if k.endswith("running_mean")}
    save("da_iter_c1", arrays, meta)

    make_da2(ref_train, BiSeNet, TinyDomainDiscriminator)

    with open(os.path.join(HERE, "state_dict_keys.json"), "w") as f:
        json.dump(keys, f)
    print("wrote state_dict_keys.json")
    make_extras(BiSeNet, DomainDiscriminator)


def make_extras(BiSeNet, DomainDiscriminator):
    """API surface beyond the C1 captures: BiSeNet with the ResNet-101 context path
    (build_contextpath.py:32-57), DomainDiscriminator(with_grl=True) (model.py:9-17, 61-62)
    and UpSampler (model.py:19-28).  Keys of the R101 model go to state_dict_keys_r101.json."""
    from models.domain_shift.adversarial.model import UpSampler
    torch.manual_seed(42)
    arrays, meta = {}, {}
    g = apply_recipe(BiSeNet(19, "resnet101"), seed=4)
    with open(os.path.join(HERE, "state_dict_keys_r101.json"), "w") as f:
        json.dump([[k, list(v.shape)] for k, v in g.state_dict().items()], f)
    x = synthetic_images(2, 64, 128, seed=49)
    y = synthetic_labels(2, 64, 128, seed=50)
    g.train()
    out, a1, a2 = g(x)
    ce = torch.nn.CrossEntropyLoss(ignore_index=19)
    loss = ce(out, y) + ce(a1, y) + ce(a2, y)
    loss.backward()
    meta["r101_loss"] = float(loss)
    for nm, t in (("r101_out", out), ("r101_aux1", a1), ("r101_aux2", a2)):
        summarize(arrays, meta, nm, t.detach())
    arrays["r101_out_argmax"] = out.detach().argmax(1).to(torch.uint8).numpy()
    param_summary(arrays, meta, "r101_grad", {k: p.grad for k, p in g.named_parameters()})
    g.eval()
    with torch.no_grad():
        summarize(arrays, meta, "r101_eval_out", g(x))

    # gradient reversal: D(with_grl=True) has the same forward and the negated, lambda-scaled
    # input gradient; its own parameter gradients are NOT reversed (the GRL sits after them)
    z = torch.randn(2, 19, 64, 128, generator=torch.Generator().manual_seed(7))
    D = apply_recipe(DomainDiscriminator(19, with_grl=True, lambda_=0.1), seed=2)
    zi = z.clone().requires_grad_(True)
    p = D(torch.softmax(zi, 1))
    l = torch.nn.BCEWithLogitsLoss()(p, torch.ones_like(p))
    l.backward()
    arrays["grl_pred"] = p.detach().numpy()
    meta["grl_loss"] = float(l)
    summarize(arrays, meta, "grl_dz", zi.grad)
    param_summary(arrays, meta, "grl_grad", {k: q.grad for k, q in D.named_parameters()})

    # UpSampler: x8 bilinear (align_corners=False) then 1x1 conv with bias
    up = apply_recipe(UpSampler(19), seed=5)
    u = torch.randn(2, 19, 16, 32, generator=torch.Generator().manual_seed(8)).requires_grad_(True)
    o = up(u)
    w = torch.randn(o.shape, generator=torch.Generator().manual_seed(9))
    (o * w).sum().backward()
    summarize(arrays, meta, "up_out", o.detach())
    summarize(arrays, meta, "up_du", u.grad)
    param_summary(arrays, meta, "up_grad", {k: q.grad for k, q in up.named_parameters()})
    save("extras", arrays, meta)


def make_da2(ref_train, BiSeNet, TinyDomainDiscriminator):
    """adversarial_train_2 (train.py:322-500): 2 epochs x 1 iteration, source images larger
    than the target (exercises adaptive_avg_pool2d), validation at epoch 1."""
    torch.manual_seed(42)
    g = apply_recipe(BiSeNet(19, "resnet18"), seed=1)
    d = apply_recipe(TinyDomainDiscriminator(19), seed=2)
    og = torch.optim.Adam(g.parameters(), lr=1e-4)
    od = torch.optim.Adam(d.parameters(), lr=1e-4, weight_decay=1e-4)
    xs = synthetic_images(2, 160, 320, seed=47)
    ys = synthetic_labels(2, 160, 320, seed=48)
    xt = synthetic_images(2, 128, 256, seed=46)
    yt = synthetic_labels(2, 128, 256, seed=43)
    cap = Capture()
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as tmp:
        os.chdir(tmp)
        try:
            ref_train.adversarial_train_2(
                iterations=1, epochs=2, generator=g, discriminator=d, generator_optimizer=og,
                discriminator_optimizer=od, source_dataloader=[(xs, ys.unsqueeze(1))],
                target_dataloader=[(xt, yt.unsqueeze(1))], generator_loss=torch.nn.CrossEntropyLoss(ignore_index=19),
                discriminator_loss=torch.nn.BCEWithLogitsLoss(), lambda_=0.1, gen_init_lr=1e-4,
                gen_power=0.9, dis_power=0.05, dis_init_lr=1e-4, lr_decay_iter=1,
                num_classes=19, class_names=[str(i) for i in range(19)],
                val_loader=[(xt, yt.unsqueeze(1))], do_validation=1, callbacks=[cap])
        finally:
            os.chdir(cwd)
    arrays, meta = {}, {"epochs": cap.epochs, "val_mIoU": float(cap.val["validation_mIoU"])}
    param_summary(arrays, meta, "gparam", dict(g.named_parameters()))
    param_summary(arrays, meta, "dparam", dict(d.named_parameters()))
    meta["g_running_mean_sum"] = {k: float(v.double().sum()) for k, v in g.state_dict().items()
                                  if k.endswith("running_mean")}
    save("da2_c1", arrays, meta)


def make_inputs():
    """The reference's input-pipeline code that needs no torchvision kernel, run on synthetic
    data: GTA5.__decode_label__ (datasets/gta5.py:111-119, colour map :10-46) on a colour image
    holding every colour of the map (ignore classes, the car / license-plate and pole /
    polegroup shared colours), near-miss and random colours; IntRangeTransformer(0, 19)
    (utils.py:67-75) on int64 and float label values; CityScapes.__merge_ids__
    (datasets/cityscapes.py:31-50) and GTA5.__make_dataset__ (datasets/gta5.py:85-100) on
    synthetic file lists (their order as a glob could return it)."""
    from datasets.cityscapes import CityScapes
    from datasets.gta5 import GTA5, cityscape_color_map, cityscape_color_map_df
    from utils import IntRangeTransformer
    g = torch.Generator().manual_seed(7)
    pal = [tuple(int(c) for c in v[1]) for v in cityscape_color_map.values()]
    train = [tuple(int(c) for c in cityscape_color_map_df.loc[cityscape_color_map_df[0] == i].iloc[0, 1])
             for i in range(19)]
    for col in train:  # one channel off by one: no match
        pal.append((min(col[0] + 1, 255), col[1], col[2]))
        pal.append((col[0], max(col[1] - 1, 0), col[2]))
    pal += [tuple(int(c) for c in torch.randint(0, 256, (3,), generator=g)) for _ in range(24)]
    pal = torch.tensor(pal, dtype=torch.long)
    h, w = 48, 80
    idx = torch.randint(0, len(pal), (h, w), generator=g)
    idx.view(-1)[:len(pal)] = torch.arange(len(pal))  # every palette colour at least once
    label = pal[idx].permute(2, 0, 1).contiguous()  # [3, H, W] long, as read_image(...).long()
    ids = GTA5.__decode_label__(None, label, cityscape_color_map_df)
    arrays = {"gta5_rgb": label.permute(1, 2, 0).to(torch.uint8).numpy(),
              "gta5_ids": ids[0].to(torch.uint8).numpy()}
    meta = {"gta5_palette": pal.tolist(), "gta5_ids_shape": list(ids.shape)}
    clamp = IntRangeTransformer(min_val=0, max_val=19)
    li = torch.randint(-40, 300, (1, 32, 48), generator=g)
    lf = torch.randn(1, 32, 48, generator=g) * 40 + 9
    arrays.update({"int_range_in_long": li.numpy().astype(np.int32), "int_range_out_long": clamp(li).numpy().astype(np.int32),
                   "int_range_in_float": lf.numpy(), "int_range_out_float": clamp(lf).numpy().astype(np.int32)})
    # Cityscapes id merge: images and gtFine annotations (colour, instance and label-id maps)
    cities = {"aachen": ["000000_000019", "000001_000019"], "bochum": ["000000_000313"],
              "zurich": ["000121_000019", "000007_000019"]}
    imgs, anns = [], []
    for city, frames in cities.items():
        for fr in frames:
            imgs.append(f"Cityscapes/images/train/{city}/{city}_{fr}_leftImg8bit.png")
            for kind in ("color", "instanceIds", "labelIds"):
                anns.append(f"Cityscapes/gtFine/train/{city}/{city}_{fr}_gtFine_{kind}.png")
    perm = torch.randperm(len(imgs), generator=g).tolist()
    imgs = [imgs[i] for i in perm]
    perm = torch.randperm(len(anns), generator=g).tolist()
    anns = [anns[i] for i in perm]
    cs = types.SimpleNamespace(images_filename=imgs, annotations_filename=anns)
    df = CityScapes.__merge_ids__(cs)
    meta["cityscapes"] = {"images": imgs, "annotations": anns,
                          "merged": [[r["path"], list(r["labels"])] for _, r in df.iterrows()]}
    gi = [f"GTA5/images/{i:05d}.png" for i in (3, 1, 10, 2, 25)]
    gl = [f"GTA5/labels/{i:05d}.png" for i in (25, 2, 3, 10, 1)]
    gt = types.SimpleNamespace(images_filenames=gi, labels_filenames=gl)
    df = GTA5.__make_dataset__(gt)
    meta["gta5_dataset"] = {"images": gi, "labels": gl,
                            "pairs": [[r["image"], list(r["label"])] for _, r in df.iterrows()]}
    save("inputs", arrays, meta)


if __name__ == "__main__":
    main()
