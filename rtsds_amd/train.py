"""Training loops -- drop-in for the reference's train.py (same function names and keyword
signatures, train.py:24-35, 130-136), running every kernel through librtsds_hip.so.

The per-iteration bodies are factored into ``seg_step`` (train.py:65-113) and ``da_step``
(train.py:172-284) so the benchmark times exactly the loop body.  Host synchronisation is
one ``.item()`` batch per iteration (losses + pixel-accuracy counter fetched together)
instead of the reference's 6-9 separate syncs; the logged values are identical.
"""
import torch

from . import functional as F
from . import losses, utils
from .callbacks import Callback
from .validation import val_GTA5

try:
    from tqdm import tqdm
except ImportError:  # pragma: no cover
    def tqdm(it, **_):
        return it


def _unpack(outputs):
    if isinstance(outputs, tuple):
        return outputs
    return outputs, None, None


def _fused_heads(model, criterion, inputs):
    """Low-res heads + shared resize geometry when the final resizes can be fused into the
    cross-entropy (the model exposes forward_lowres, the criterion is the unweighted-mean CE,
    all heads share one upsample geometry), else None."""
    if not (isinstance(criterion, losses.CrossEntropyLoss) and hasattr(model, "forward_lowres")):
        return None
    heads = model.forward_lowres(inputs)
    geos = {geo for _, geo in heads}
    if len(geos) != 1 or None in geos:
        return [F.interpolate_geometry(t, geo) if geo is not None else t for t, geo in heads], None
    geo = geos.pop()
    ts = [t for t, _ in heads]
    if not F.upsample_cross_entropy_supported(ts, geo, criterion.ignore_index):
        return [F.interpolate_geometry(t, geo) for t in ts], None
    return ts, geo


def seg_step(model, criterion, optimizer, inputs, targets):
    """One train.train iteration body: zero_grad, forward, CE(main)+CE(aux1)+CE(aux2),
    backward, optimizer step, device-side pixel-accuracy count.  Returns device tensors
    (loss, correct) -- no host sync.  When the model exposes its pre-resize heads, the
    bilinear resizes, the three cross-entropies and the accuracy argmax run as one fused
    kernel (functional.upsample_cross_entropy) -- same losses and gradients, no
    full-resolution logits."""
    optimizer.zero_grad()
    fused = _fused_heads(model, criterion, inputs)
    if fused is not None and fused[1] is not None:
        correct = torch.zeros(1, dtype=torch.int64, device=fused[0][0].device)
        loss = F.upsample_cross_entropy(fused[0], targets, fused[1], criterion.ignore_index, correct)
        loss.backward()
        optimizer.step()
        return loss.detach(), correct
    if fused is not None:
        outs = list(fused[0]) + [None] * (3 - len(fused[0]))
        main_output, aux1, aux2 = outs[:3]
    else:
        main_output, aux1, aux2 = _unpack(model(inputs))
    loss = criterion(main_output, targets)
    if aux1 is not None:
        loss = loss + criterion(aux1, targets)
    if aux2 is not None:
        loss = loss + criterion(aux2, targets)
    loss.backward()
    optimizer.step()
    correct = torch.zeros(1, dtype=torch.int64, device=main_output.device)
    F.argmax_channels(main_output.detach(), targets, correct, want_map=False)
    return loss.detach(), correct


def train(epoch: int, model: torch.nn.Module, train_loader, criterion: torch.nn.Module,
          optimizer: torch.optim.Optimizer, init_lr: float, max_iter: int, power: float = 0.9,
          lr_decay_iter: float = 1.0, device: str = "cuda", callbacks: list = []):
    """One epoch of segmentation training (train.py:24-128)."""
    for cb in callbacks:
        cb.on_train_begin()
    model.train()
    running_loss, correct, total = 0.0, 0, 0
    for batch_idx, (inputs, targets) in tqdm(enumerate(train_loader), total=len(train_loader),
                                             desc=f"Epoch {epoch + 1}", leave=False):
        current_iter = epoch * len(train_loader) + batch_idx
        if current_iter % lr_decay_iter == 0 and current_iter <= max_iter:
            utils.poly_lr_scheduler(optimizer, init_lr, current_iter, lr_decay_iter, max_iter, power)
        inputs = inputs.to(device)
        targets = targets.to(device).squeeze(1)
        loss, corr = seg_step(model, criterion, optimizer, inputs, targets)
        vals = torch.stack([loss.double(), corr[0].double()]).tolist()
        running_loss += vals[0]
        total += targets.size(0) * targets.size(1) * targets.size(2)
        correct += int(vals[1])
        for cb in callbacks:
            cb.on_batch_end(batch_idx, {"train_loss": vals[0],
                                        "train_accuracy": 100.0 * correct / total})
    train_loss = running_loss / len(train_loader)
    train_accuracy = 100.0 * correct / total
    print(f"Train Epoch: {epoch + 1} Loss: {train_loss:.6f} Acc: {train_accuracy:.2f}%")
    for cb in callbacks:
        cb.on_epoch_end(epoch, {"train_loss": train_loss, "train_accuracy": train_accuracy})
    return model


def da_step(generator, discriminator, generator_optimizer, discriminator_optimizer,
            generator_loss, discriminator_loss, source_image, source_label, target_image,
            lambda_, iterations):
    """One adversarial_train iteration body (train.py:174-275, LR scheduling excluded).
    Returns device tensors (l_seg, l_adv, l_dsrc, l_dtgt, correct)."""
    generator_optimizer.zero_grad()
    discriminator_optimizer.zero_grad()
    # the discriminator is frozen while the generator trains (train.py:192-193)
    for p in discriminator.parameters():
        p.requires_grad = False
    out = generator(source_image)
    if isinstance(out, tuple):
        loss_seg = generator_loss(out[0], source_label)
        for aux in out[1:]:
            if aux is not None:  # DeepLab returns (x, None, None) (deeplabv2.py:128-129)
                loss_seg = loss_seg + generator_loss(aux, source_label)
        source_features = out[0]
    else:
        loss_seg = generator_loss(out, source_label)
        source_features = out
    loss_seg = loss_seg / iterations
    loss_seg.backward()

    tout = generator(target_image)
    target_feature = tout[0] if isinstance(tout, tuple) else tout
    pred_t = discriminator(F.softmax(target_feature, dim=1))
    ones = torch.ones(pred_t.size(), device=pred_t.device)
    loss_adv = lambda_ * discriminator_loss(pred_t, ones) / iterations
    loss_adv.backward()

    for p in discriminator.parameters():
        p.requires_grad = True
    source_features = source_features.detach()
    target_feature = target_feature.detach()
    pred_s = discriminator(F.softmax(source_features, dim=1))
    loss_dsrc = discriminator_loss(pred_s, torch.ones(pred_s.size(), device=pred_s.device)) / iterations
    loss_dsrc.backward()
    pred_t2 = discriminator(F.softmax(target_feature, dim=1))
    loss_dtgt = discriminator_loss(pred_t2, torch.zeros(pred_t2.size(), device=pred_t2.device)) / iterations
    loss_dtgt.backward()

    generator_optimizer.step()
    discriminator_optimizer.step()
    correct = torch.zeros(1, dtype=torch.int64, device=source_features.device)
    F.argmax_channels(source_features, source_label, correct, want_map=False)
    return loss_seg.detach(), loss_adv.detach(), loss_dsrc.detach(), loss_dtgt.detach(), correct


def adversarial_train(iterations: int, epochs: int, generator: torch.nn.Module,
                      discriminator: torch.nn.Module, generator_optimizer, discriminator_optimizer,
                      source_dataloader, target_dataloader, generator_loss: torch.nn.Module,
                      discriminator_loss: torch.nn.Module, lambda_: float, gen_init_lr: float,
                      gen_power: float, dis_power: float, dis_init_lr: float, lr_decay_iter: float,
                      num_classes: int, class_names: list, val_loader, do_validation: int = 1,
                      device: str = "cuda", when_print: int = 10, callbacks: list = []):
    """AdaptSegNet-style output-space adversarial training (train.py:130-318)."""
    gen_lr = None
    for epoch in range(epochs):
        for cb in callbacks:
            cb.on_train_begin()
        run = [0.0, 0.0, 0.0, 0.0]
        g_correct, g_total = 0, 0
        best_mIoU = 0
        generator.train()
        discriminator.train()
        dis_lr = utils.poly_lr_scheduler(discriminator_optimizer, dis_init_lr, epoch, lr_decay_iter,
                                         epochs, dis_power)
        max_iter = epochs * iterations
        for i in tqdm(range(iterations), total=iterations, desc=f"Epoch {epoch}"):
            current_iter = epoch * iterations + i
            if current_iter % lr_decay_iter == 0 and current_iter <= max_iter:
                gen_lr = utils.poly_lr_scheduler(generator_optimizer, gen_init_lr, current_iter,
                                                 lr_decay_iter, max_iter, gen_power)
            source_image, source_label = next(iter(source_dataloader))
            target_image, _ = next(iter(target_dataloader))
            source_image, source_label = source_image.to(device), source_label.to(device)
            source_label = source_label.squeeze(1)
            target_image = target_image.to(device)
            *losses, corr = da_step(generator, discriminator, generator_optimizer,
                                    discriminator_optimizer, generator_loss, discriminator_loss,
                                    source_image, source_label, target_image, lambda_, iterations)
            vals = torch.stack([l.double() for l in losses] + [corr[0].double()]).tolist()
            for k in range(4):
                run[k] += vals[k]
            g_correct += int(vals[4])
            g_total += source_label.size(0) * source_label.size(1) * source_label.size(2)
            for cb in callbacks:
                cb.on_batch_end(i, {"loss_gen_source": vals[0], "loss_adversarial": vals[1],
                                    "loss_disc_source": vals[2], "loss_disc_target": vals[3]})
        print(f"Epoch Results {epoch}")
        utils.tabular_print({
            "loss_gen_source": run[0] / iterations, "loss_adversarial": run[1] / iterations,
            "loss_disc_source": run[2] / iterations, "loss_disc_target": run[3] / iterations,
            "Genrator Accuracy": (100.0 * g_correct / g_total),
            "dis_lr": dis_lr if dis_lr else -1, "gen_lr": gen_lr if gen_lr else -1})
        for cb in callbacks:
            cb.on_epoch_end(epoch, {"dis_lr": dis_lr if dis_lr else -1,
                                    "gen_lr": gen_lr if gen_lr else -1,
                                    "Genrator Accuracy": 100.0 * g_correct / g_total})
        if do_validation != 0 and epoch % do_validation == 0:
            print("-" * 50, "Validation", "-" * 50)
            validation_mIou, _ = val_GTA5(epoch, generator, val_loader, num_classes, class_names,
                                          callbacks, device=device)
            print("-" * 100)
            if validation_mIou > best_mIoU:
                best_mIoU = validation_mIou
                torch.save(generator.state_dict(), "best_generator.pth")
                torch.save(discriminator.state_dict(), "best_discriminator.pth")
                print(f"Best Model Saved at Epoch {epoch}")
    for cb in callbacks:
        cb.on_train_end()


__all__ = ["train", "adversarial_train", "seg_step", "da_step", "Callback"]
