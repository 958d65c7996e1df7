"""CLI entry -- drop-in for the reference's main.py (flags main.py:233-260, config via
config.yaml, factories main.py:110-231, dispatch main.py:272-374) on the HIP path.

    python -m rtsds_amd.main [--config rtsds_amd/config.yaml] [--domain_adaptation]
                             [--model bisenet|deeplab] [--dataset cityscapes|gta5] [--seed 42]
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m rtsds_amd.main --domain_adaptation

Datasets (main.py:46-108): when the configured directories exist, the reference's readers
(rtsds_amd.datasets) feed the device-side transforms (rtsds_amd.transforms: antialiased
resize, normalize, augmentation, label clamp as HIP kernels); otherwise synthetic loaders of
the configured shapes are used (ImageNet-normalised 0-255 images, labels 0..19 with
19 = ignore), sharded per rank.  Deviations from the reference (documented in DESIGN.md): DA accepts a
DeepLab generator; validation accepts class_names / detailed_report.
"""
import argparse
import os
from collections import namedtuple

import numpy as np
import torch
import yaml

from . import losses, optim
from .models.bisenet import build_bisenet
from .models.deeplabv2 import deeplabv2
from .models.domain_shift.adversarial.model import DomainDiscriminator, TinyDomainDiscriminator
from .runtime import set_compute_dtype
from .train import adversarial_train, train
from .utils import dist_env, forModel
from .validation import val, val_GTA5


def optimzer_loss_loader(model, optimizer_config, loss_config):
    """main.py:110-136 with the HIP-backed Adam / SGD and losses."""
    if optimizer_config["name"] == "Adam":
        optimizer = optim.Adam(model.parameters(), lr=optimizer_config["lr"],
                               weight_decay=optimizer_config.get("weight_decay", 0))
    elif optimizer_config["name"] == "SGD":
        optimizer = optim.SGD(model.parameters(), lr=optimizer_config["lr"],
                              momentum=optimizer_config["momentum"])
    else:
        raise ValueError("Invalid optimizer name. Please select Adam or SGD")
    if loss_config["name"] == "CrossEntropy":
        loss = losses.CrossEntropyLoss(ignore_index=loss_config.get("ignore_index"))
    elif loss_config["name"] == "BCEWithLogits":
        loss = losses.BCEWithLogitsLoss()
    else:
        raise ValueError("Invalid loss name. Please select CrossEntropy or BCEWithLogits")
    return optimizer, loss


def _generator(model_cfg, name):
    if name == "bisenet":
        b = model_cfg["bisenet"]
        return build_bisenet.BiSeNet(num_classes=b["num_classes"], context_path=b["backbone"])
    if name == "deeplab":
        d = model_cfg["deeplab"]
        return deeplabv2.get_deeplab_v2(d["num_classes"], pretrain=d.get("pretrain", False),
                                        pretrain_model_path=d.get("pretrain_model_path"))
    raise ValueError("Invalid model name. Please select deeplab or bisenet")


def model_loader(config, is_adversarial, model_name):
    """main.py:138-231.  Models are moved to the device BEFORE the optimizers are built so
    the fused Adam's arena is created on the GPU."""
    model_cfg = config.model
    if is_adversarial:
        adv = model_cfg["adversarial_model"]
        gen = forModel(_generator(model_cfg, adv["generator"]["name"]), config.device)
        g_opt, g_loss = optimzer_loss_loader(gen, adv["generator"]["optimizer"], adv["generator"]["criterion"])
        g_hp = {"gen_init_lr": adv["generator"]["optimizer"]["lr"], "gen_power": adv["generator"]["power_lr_factor"]}
        dcfg = adv["discriminator"]
        dis = (TinyDomainDiscriminator(num_classes=dcfg["input_channels"]) if dcfg["name"] == "tiny"
               else DomainDiscriminator(num_classes=dcfg["input_channels"]))
        dis = forModel(dis, config.device)
        d_opt, d_loss = optimzer_loss_loader(dis, dcfg["optimizer"], dcfg["criterion"])
        d_hp = {"dis_init_lr": dcfg["optimizer"]["lr"], "dis_power": dcfg["power_lr_factor"]}
        return (gen, g_opt, g_loss, g_hp), (dis, d_opt, d_loss, d_hp)
    cfg = model_cfg["deeplab" if model_name == "deeplab" else "bisenet"]
    model = forModel(_generator(model_cfg, model_name), config.device)
    opt, loss = optimzer_loss_loader(model, cfg["optimizer"], cfg["criterion"])
    return model, opt, loss, {"init_lr": cfg["optimizer"]["lr"], "power": cfg["power_lr_factor"]}


class SyntheticLoader:
    """Fixed synthetic batches of the configured size (list semantics: len / iter / index)."""

    def __init__(self, batches, batch_size, size, num_classes, seed):
        h, w = size
        g = torch.Generator().manual_seed(seed)
        mean = torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)
        std = torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)
        self.data = []
        for _ in range(batches):
            x = (torch.randint(0, 256, (batch_size, 3, h, w), generator=g).float() - mean) / std
            y = torch.randint(0, num_classes + 1, (batch_size, 1, h, w), generator=g)
            self.data.append((x, y))

    def __len__(self):
        return len(self.data)

    def __iter__(self):
        return iter(self.data)


def real_datasets_loader(config, is_augmented, device="cuda"):
    """main.py:60-108 on the device pipeline: the reference's readers (PNG decode on CPU
    DataLoader workers) deliver raw uint8 samples, batches go to HBM and through the
    torchvision-equivalent HIP transforms (rtsds_amd.transforms); under data parallelism each
    rank reads a disjoint shard of the training sets (DistributedSampler, a new permutation per
    iterator -- transforms.DeviceLoader advances its epoch); validation reads the whole set."""
    from torch.utils.data import DataLoader
    from torch.utils.data.distributed import DistributedSampler

    from . import transforms as T
    from .datasets import GTA5, CityScapes
    cs, gta = config.data["cityscapes"], config.data["gta5_modified"]
    cs_size, gta_size = T.parse_size(cs["image_size"]), T.parse_size(gta["image_size"])
    rank, _, world = dist_env()

    def loader(ds, bs, workers, shuffle, shard=True):
        sampler = DistributedSampler(ds, num_replicas=world, rank=rank, shuffle=shuffle) \
            if world > 1 and shard else None
        return DataLoader(ds, batch_size=bs, shuffle=shuffle and sampler is None, sampler=sampler, pin_memory=False,
                          num_workers=workers, collate_fn=T.collate_raw)

    city_img = T.ImagePipeline(cs_size)
    city_lbl = T.LabelPipeline(cs_size, clamp=(0, cs["num_classes"]))
    gta_img = T.ImagePipeline(gta_size, augment=T.augmentation_loader(config, 0.5) if is_augmented else None)
    gta_lbl = T.LabelPipeline(gta_size)
    train_ds = CityScapes(cs["segmentation_train_dir"], cs["images_train_dir"])
    val_ds = CityScapes(cs["segmentation_val_dir"], cs["images_val_dir"])
    gta_ds = GTA5(gta["images_dir"], gta["segmentation_dir"], None, None)
    return (T.DeviceLoader(loader(train_ds, cs["batch_size"], cs["num_workers"], True), city_img, city_lbl, device),
            # validation is not sharded: a DistributedSampler pads shards with duplicates and
            # the confusion histogram is per process, so every rank evaluates the full val set
            # and reports the reference's full-set mIoU
            T.DeviceLoader(loader(val_ds, cs["batch_size"], cs["num_workers"], False, shard=False),
                           city_img, city_lbl, device),
            T.DeviceLoader(loader(gta_ds, gta["batch_size"], gta["num_workers"], True), gta_img, gta_lbl, device))


def datasets_loader(config, is_augmented):
    """main.py:60-108: the dataset directories of config.yaml through the device pipeline when
    they exist, else synthetic loaders of the configured shapes."""
    cs, gta = config.data["cityscapes"], config.data["gta5_modified"]
    present = os.path.isdir(cs["images_train_dir"]) and os.path.isdir(gta["images_dir"])
    if present:
        return real_datasets_loader(config, is_augmented, config.device)
    rank = dist_env()[0]
    nb = config.data.get("synthetic_batches", 4)
    size = lambda s: [int(v) for v in str(s).split(",")]  # noqa: E731
    city = SyntheticLoader(nb, cs["batch_size"], size(cs["image_size"]), cs["num_classes"], 1000 + 2 * rank)
    val_l = SyntheticLoader(1, cs["batch_size"], size(cs["image_size"]), cs["num_classes"], 7)
    gta5 = SyntheticLoader(nb, gta["batch_size"], size(gta["image_size"]), gta["num_classes"], 2000 + 2 * rank)
    return city, val_l, gta5


def argumnet_parser(argv=None):
    p = argparse.ArgumentParser(description="Semantic Segmentation and Domain Adaptation (MI355X)")
    p.add_argument("--config", type=str, default=os.path.join(os.path.dirname(__file__), "config.yaml"))
    p.add_argument("--dataset", type=str, default="cityscapes")
    p.add_argument("--augmented", action="store_true")
    p.add_argument("--domain_adaptation", action="store_true")
    p.add_argument("--model", type=str, default="bisenet")
    p.add_argument("--wandb", action="store_true")
    p.add_argument("--seed", type=int, default=42)
    return p.parse_args(argv)


def set_seed(seed):
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)
    np.random.seed(seed)


def load_config(path):
    with open(path) as f:
        cfg = yaml.safe_load(f)
    return namedtuple("Config", cfg.keys())(*cfg.values())


def main(argv=None):
    args = argumnet_parser(argv)
    set_seed(args.seed)
    config = load_config(args.config)
    set_compute_dtype(torch.bfloat16 if getattr(config, "precision", "fp32") == "bf16" else torch.float32)
    train_dl, val_dl, gta_dl = datasets_loader(config, args.augmented)
    callbacks = []
    if args.domain_adaptation:
        (g, g_opt, g_loss, g_hp), (d, d_opt, d_loss, d_hp) = model_loader(config, True, args.model)
        t = config.training["domain_adaptation"]
        adversarial_train(iterations=t["iterations"], epochs=t["epochs"], lambda_=t["lambda"], generator=g,
                          discriminator=d, generator_optimizer=g_opt, discriminator_optimizer=d_opt,
                          generator_loss=g_loss, discriminator_loss=d_loss, source_dataloader=gta_dl,
                          target_dataloader=train_dl, gen_init_lr=g_hp["gen_init_lr"],
                          dis_init_lr=d_hp["dis_init_lr"], lr_decay_iter=t["lr_decay_iter"],
                          gen_power=g_hp["gen_power"], dis_power=d_hp["dis_power"],
                          num_classes=t["num_classes"], class_names=config.meta["class_names"],
                          val_loader=val_dl, do_validation=t["do_validation"], when_print=t["when_print"],
                          callbacks=callbacks, device=config.device)
    else:
        if args.dataset == "gta5":
            train_dl = gta_dl
        model, opt, crit, hp = model_loader(config, False, args.model)
        t = config.training["segmentation"]
        max_iter = t["epochs"] * len(train_dl)
        for epoch in range(t["epochs"]):
            train(model=model, optimizer=opt, criterion=crit, train_loader=train_dl, epoch=epoch,
                  init_lr=hp["init_lr"], lr_decay_iter=t["lr_decay_iter"], power=hp["power"],
                  max_iter=max_iter, callbacks=callbacks, device=config.device)
            val(epoch=epoch, model=model, val_loader=val_dl, num_classes=t["num_classes"],
                class_names=config.meta["class_names"], detailed_report=True, device=config.device,
                callbacks=callbacks)


if __name__ == "__main__":
    main()
