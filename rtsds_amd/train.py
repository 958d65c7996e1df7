"""Training loops -- drop-in for the reference's train.py (same function names and keyword
signatures, train.py:24-35, 130-136), running every kernel through librtsds_hip.so.

The per-iteration bodies are factored into ``seg_step`` (train.py:65-113) and ``da_step``
(train.py:172-284) so the benchmark times exactly the loop body.  Host synchronisation is
one ``.item()`` batch per iteration (losses + pixel-accuracy counter fetched together)
instead of the reference's 6-9 separate syncs; the logged values are identical.
"""
import contextlib

import torch

from . import functional as F
from . import losses, utils
from .optim import begin_grad_phase
from .runtime import branch_stream, branches_enabled, branches_serial, collect_cuts, dp_world
from .callbacks import Callback
from .validation import val_GTA5

try:
    from tqdm import tqdm
except ImportError:  # pragma: no cover
    def tqdm(it, **_):
        return it


def _host_values(tensors):
    """The iteration's logged scalars in one host sync.  Under data parallelism each rank
    holds its contribution to the global-batch losses (and its pixel count), so they are
    summed over ranks first."""
    t = torch.stack([x.double().reshape(()) for x in tensors])
    if dp_world() > 1:
        import torch.distributed as dist
        dist.all_reduce(t)
    return t.tolist()


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


_ONES = {}


def _one(t):
    """The unit seed of ``t.backward()`` as a cached tensor: autograd's own ones_like is a fill
    launch per backward (a node of every replay of a captured step)."""
    key = (t.device, t.dtype, tuple(t.shape))
    one = _ONES.get(key)
    if one is None:
        one = _ONES[key] = torch.ones_like(t)
    return one


def _backward(loss, optimizer, cuts, since=None):
    """loss.backward(); with cuts (runtime.grad_cut under data parallelism, recorded in forward
    order): phase 1 down to the last cut's leaf, then, cut by cut from the last, the all-reduce
    of the gradients complete so far is started and the backward continues through that cut
    tensor down to the previous cut's leaf -- one gradient bucket per phase, each reducing
    while the next phase computes.  Same gradients (a cut leaf accumulates exactly what its
    tensor would have received).  ``since``: the gradient-arrival generation of this backward
    (optim.begin_grad_phase) when an earlier backward already touched the parameters."""
    loss.backward(_one(loss))
    for x, xd in reversed(cuts or []):
        optimizer.start_grad_allreduce(partial=True, since=since)
        if xd.grad is not None:
            torch.autograd.backward([x], [xd.grad])


def seg_step(model, criterion, optimizer, inputs, targets):
    """One train.train iteration body: zero_grad, forward, CE(main)+CE(aux1)+CE(aux2),
    backward, optimizer step, device-side pixel-accuracy count.  Returns device tensors
    (loss, correct) -- no host sync.  When the model exposes its pre-resize heads, the
    bilinear resizes, the three cross-entropies and the accuracy argmax run as one fused
    kernel (functional.upsample_cross_entropy) -- same losses and gradients, no
    full-resolution logits."""
    optimizer.zero_grad()
    # data parallelism: the backward runs in two phases split at the models' grad_cut tensor,
    # and the all-reduce of the first phase's (late layers') gradients overlaps the second
    split = dp_world() > 1 and hasattr(optimizer, "start_grad_allreduce")
    with collect_cuts(split) as cuts:
        fused = _fused_heads(model, criterion, inputs)
        if fused is None:
            outs = _unpack(model(inputs))
    if fused is not None and fused[1] is not None:
        correct = torch.empty(1, dtype=torch.int64, device=fused[0][0].device)  # (overwritten)
        loss = F.upsample_cross_entropy(fused[0], targets, fused[1], criterion.ignore_index, correct, set_correct=True)
        _backward(loss, optimizer, cuts)
        optimizer.step()
        return loss.detach(), correct
    if fused is not None:
        outs = list(fused[0]) + [None] * (3 - len(fused[0]))
        main_output, aux1, aux2 = outs[:3]
    else:
        main_output, aux1, aux2 = outs
    loss = criterion(main_output, targets)
    if aux1 is not None:
        loss = loss + criterion(aux1, targets)
    if aux2 is not None:
        loss = loss + criterion(aux2, targets)
    _backward(loss, optimizer, cuts)
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
        vals = _host_values([loss, corr[0]])
        running_loss += vals[0]
        total += targets.size(0) * targets.size(1) * targets.size(2) * dp_world()
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


def _main_output(model, x):
    """The model's main (first) output at full resolution; auxiliary heads that the caller
    would discard are not computed when the model exposes forward_lowres (they hold no state)."""
    if hasattr(model, "forward_lowres"):
        (t, geo), = model.forward_lowres(x, main_only=True)
        return F.interpolate_geometry(t, geo) if geo is not None else t
    out = model(x)
    return out[0] if isinstance(out, tuple) else out


def _seg_loss(model, criterion, x, label, correct):
    """Sum over the model's heads of criterion(head, label) (train.py:86-92, 196-204, 392-399)
    plus head 0's pixel matches added to ``correct``.  Returns (loss, low-res main head and its
    resize geometry, or the full-resolution main output with geometry None)."""
    fused = _fused_heads(model, criterion, x)
    if fused is not None and fused[1] is not None:
        heads, geo = fused
        loss = F.upsample_cross_entropy(heads, label, geo, criterion.ignore_index, correct)
        return loss, heads[0], geo
    if fused is not None:
        outs = fused[0]
    else:
        out = model(x)
        outs = list(out) if isinstance(out, tuple) else [out]
    loss = None
    for o in outs:
        if o is None:  # DeepLab returns (x, None, None) (deeplabv2.py:128-129)
            continue
        l = criterion(o, label)
        loss = l if loss is None else loss + l
    F.argmax_channels(outs[0].detach(), label, correct, want_map=False)
    return loss, outs[0], None


# da_step (fused path, single process): target forward on a second stream during the source
# backward (see _da_step_fused); False = strictly serial issue (A/B tests)
DA_OVERLAP = True


def _start_allreduce(optimizer):
    if dp_world() > 1 and hasattr(optimizer, "start_grad_allreduce"):
        optimizer.start_grad_allreduce()


def _full(t, geo):
    return F.interpolate_geometry(t, geo) if geo is not None else t


def da_step(generator, discriminator, generator_optimizer, discriminator_optimizer,
            generator_loss, discriminator_loss, source_image, source_label, target_image,
            lambda_, iterations):
    """One adversarial_train iteration body (train.py:174-275, LR scheduling excluded).
    Returns device tensors (l_seg, l_adv, l_dsrc, l_dtgt, correct).  The source heads' resizes
    run fused into their cross-entropy; the discriminator consumes the detached main output,
    so it is resized without a gradient graph."""
    generator_optimizer.zero_grad()
    discriminator_optimizer.zero_grad()
    # the discriminator is frozen while the generator trains (train.py:192-193)
    for p in discriminator.parameters():
        p.requires_grad = False
    correct = torch.zeros(1, dtype=torch.int64, device=source_image.device)
    loss_seg, main, geo = _seg_loss(generator, generator_loss, source_image, source_label, correct)
    loss_seg = loss_seg / iterations
    if geo is not None and getattr(discriminator, "accepts_padded_probs", False) and \
            hasattr(generator, "forward_lowres") and main.shape[1] <= 32:
        return _da_step_fused(generator, discriminator, generator_optimizer, discriminator_optimizer,
                              discriminator_loss, main, geo, target_image, lambda_, iterations, loss_seg,
                              correct)
    loss_seg.backward(_one(loss_seg))
    with torch.no_grad():
        source_features = _full(main.detach(), geo)

    split = dp_world() > 1 and hasattr(generator_optimizer, "start_grad_allreduce")
    with collect_cuts(split) as cuts:
        target_feature = _main_output(generator, target_image)
    pred_t = discriminator(F.softmax(target_feature, dim=1))
    ones = torch.ones(pred_t.size(), device=pred_t.device)
    loss_adv = lambda_ * discriminator_loss(pred_t, ones) / iterations
    # the adversarial backward in bucketed phases at the generator's cuts (each bucket's
    # all-reduce overlaps the next phase); the rest of G's gradients are final after it and
    # their all-reduce overlaps the D phase
    _backward(loss_adv, generator_optimizer, cuts, since=begin_grad_phase() if split else None)
    _start_allreduce(generator_optimizer)

    for p in discriminator.parameters():
        p.requires_grad = True
    target_feature = target_feature.detach()
    pred_s = discriminator(F.softmax(source_features, dim=1))
    loss_dsrc = discriminator_loss(pred_s, torch.ones(pred_s.size(), device=pred_s.device)) / iterations
    loss_dsrc.backward(_one(loss_dsrc))
    pred_t2 = discriminator(F.softmax(target_feature, dim=1))
    loss_dtgt = discriminator_loss(pred_t2, torch.zeros(pred_t2.size(), device=pred_t2.device)) / iterations
    loss_dtgt.backward(_one(loss_dtgt))
    _start_allreduce(discriminator_optimizer)  # overlaps G's optimizer step

    generator_optimizer.step()
    discriminator_optimizer.step()
    return loss_seg.detach(), loss_adv.detach(), loss_dsrc.detach(), loss_dtgt.detach(), correct


def _da_step_fused(generator, discriminator, generator_optimizer, discriminator_optimizer,
                   discriminator_loss, main, geo, target_image, lambda_, iterations, loss_seg, correct):
    """da_step's discriminator phases with the full-resolution resize and softmax of each
    head fused into one pass that writes the discriminator's padded input
    (functional.upsample_softmax): identical values to softmax(interpolate(head)) -- the
    reference's D(softmax(G(x))) at train.py:225,245,256 -- without the full-resolution logits,
    the separate softmax pass or the conv's channel-pad pass.  softmax(target_feature.detach())
    (train.py:256) equals the G-phase target probabilities, so they are computed once."""
    amb = torch.cuda.current_stream(main.device)
    overlap = DA_OVERLAP and dp_world() <= 1 and branches_enabled()
    if overlap:
        # the target forward (G, resize + softmax, frozen D, loss) depends only on parameters
        # the source backward does not touch: it runs on a second stream, concurrently with
        # loss_seg.backward() (BatchNorm running statistics still update source then target;
        # the adversarial backward, on the target ops' stream, starts after the source backward
        # -- autograd orders it after the ambient stream -- so G's gradient accumulation order
        # is unchanged)
        side = branch_stream(main.device, "da_target")
        side.wait_stream(amb)
        target_image.record_stream(side)
        ctx = torch.cuda.stream(side)
    else:
        loss_seg.backward(_one(loss_seg))
        ctx = contextlib.nullcontext()
    split = dp_world() > 1 and hasattr(generator_optimizer, "start_grad_allreduce")
    with ctx, (branches_serial() if overlap else contextlib.nullcontext()), collect_cuts(split) as cuts:
        (t_low, t_geo), = generator.forward_lowres(target_image, main_only=True)
        target_probs = F.upsample_softmax(t_low, t_geo)
        pred_t = discriminator(target_probs)
        ones = torch.ones(pred_t.size(), device=pred_t.device)
        loss_adv = lambda_ * discriminator_loss(pred_t, ones) / iterations
    if overlap:
        loss_seg.backward(_one(loss_seg))
        amb.wait_stream(side)
        for t in (target_probs, loss_adv):
            t.record_stream(amb)
    with torch.no_grad():
        source_probs = F.upsample_softmax(main.detach(), geo)
    if overlap:
        # D's source phase needs only source_probs and D's (unchanged) weights, and writes only
        # D's gradients, which the adversarial backward (through the frozen D into G) never
        # touches: it runs on a third stream beside that backward; D's target phase follows it
        # (D's gradient accumulation order source -> target is kept)
        side2 = branch_stream(main.device, "da_disc")
        side2.wait_stream(amb)
        source_probs.record_stream(side2)
    _backward(loss_adv, generator_optimizer, cuts, since=begin_grad_phase() if split else None)
    _start_allreduce(generator_optimizer)

    for p in discriminator.parameters():
        p.requires_grad = True
    with torch.cuda.stream(side2) if overlap else contextlib.nullcontext():
        pred_s = discriminator(source_probs)
        loss_dsrc = discriminator_loss(pred_s, torch.ones(pred_s.size(), device=pred_s.device)) / iterations
        loss_dsrc.backward(_one(loss_dsrc))
    if overlap:
        amb.wait_stream(side)  # the adversarial backward ran on the target ops' streams
        amb.wait_stream(side2)
        loss_dsrc.record_stream(amb)
    pred_t2 = discriminator(F.detach_padded(target_probs))
    loss_dtgt = discriminator_loss(pred_t2, torch.zeros(pred_t2.size(), device=pred_t2.device)) / iterations
    loss_dtgt.backward(_one(loss_dtgt))
    _start_allreduce(discriminator_optimizer)

    generator_optimizer.step()
    discriminator_optimizer.step()
    return loss_seg.detach(), loss_adv.detach(), loss_dsrc.detach(), loss_dtgt.detach(), correct


def da2_step(generator, discriminator, generator_optimizer, discriminator_optimizer,
             generator_loss, discriminator_loss, source_image, source_label, target_image,
             lambda_adv):
    """One adversarial_train_2 iteration body (train.py:373-466, LR scheduling excluded):
    G step on L_seg(source) + lambda_adv * BCE(D(softmax(pool(G(target)))), 0), then a D step
    on BCE(D(softmax(pool(G(target)))), 1) + BCE(D(softmax(pool(G(source)))), 0) with both
    generator outputs recomputed under no_grad (train mode).  pool = adaptive_avg_pool2d to
    the target size.  D's parameter gradients of the G step are discarded by the reference
    (zero_grad before the D step), so D is frozen there.  Returns device tensors (l_seg,
    l_adv, g_total, d_real, d_fake, d_total, correct)."""
    th, tw = int(target_image.shape[2]), int(target_image.shape[3])
    b = int(target_image.shape[0])
    dev = target_image.device
    real_labels = torch.ones(b, 1, 1, 1, device=dev)
    fake_labels = torch.zeros(b, 1, 1, 1, device=dev)

    generator_optimizer.zero_grad()
    for p in discriminator.parameters():
        p.requires_grad = False
    correct = torch.zeros(1, dtype=torch.int64, device=dev)
    g_loss_seg, _, _ = _seg_loss(generator, generator_loss, source_image, source_label, correct)
    real_seg = F.adaptive_avg_pool2d(_main_output(generator, target_image), (th, tw))
    d_real_output = discriminator(F.softmax(real_seg, dim=1))
    loss_adv = discriminator_loss(d_real_output, fake_labels)
    g_loss = g_loss_seg + lambda_adv * loss_adv
    g_loss.backward(_one(g_loss))
    generator_optimizer.step()
    for p in discriminator.parameters():
        p.requires_grad = True

    discriminator_optimizer.zero_grad()
    with torch.no_grad():
        fake_seg = F.adaptive_avg_pool2d(_main_output(generator, source_image), (th, tw))
        real_seg = F.adaptive_avg_pool2d(_main_output(generator, target_image), (th, tw))
    d_real_output = discriminator(F.softmax(real_seg, dim=1))
    d_fake_output = discriminator(F.softmax(fake_seg, dim=1))
    d_real_loss = discriminator_loss(d_real_output, real_labels)
    d_fake_loss = discriminator_loss(d_fake_output, fake_labels)
    d_loss = d_real_loss + d_fake_loss
    d_loss.backward(_one(d_loss))
    discriminator_optimizer.step()
    return (g_loss_seg.detach(), loss_adv.detach(), g_loss.detach(), d_real_loss.detach(),
            d_fake_loss.detach(), d_loss.detach(), correct)


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
            vals = _host_values(list(losses) + [corr[0]])
            for k in range(4):
                run[k] += vals[k]
            g_correct += int(vals[4])
            g_total += source_label.size(0) * source_label.size(1) * source_label.size(2) * dp_world()
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


def adversarial_train_2(iterations: int, epochs: int, generator: torch.nn.Module,
                        discriminator: torch.nn.Module, generator_optimizer, discriminator_optimizer,
                        source_dataloader, target_dataloader, generator_loss: torch.nn.Module,
                        discriminator_loss: torch.nn.Module, lambda_: float, gen_init_lr: float,
                        gen_power: float, dis_power: float, dis_init_lr: float,
                        lr_decay_iter: float, num_classes: int, class_names: list, val_loader,
                        do_validation: int = 1, device: str = "cuda", when_print: int = 10,
                        callbacks: list = []):
    """Second adversarial loop (train.py:322-500): D trained on real (target) vs fake (source)
    segmentations pooled to the target size, inverted adversarial label, lambda schedule
    max(lambda, 10 lambda - 0.001 epoch).  Reference behaviour kept: both learning rates use
    ``dis_power`` (train.py:385-386), best-mIoU is reset every epoch, validation skips
    epoch 0."""
    dis_lr = gen_lr = None
    for epoch in range(epochs):
        generator.train()
        discriminator.train()
        run = {"loss_gen_source": 0.0, "loss_adversarial": 0.0, "loss_gen_total": 0.0,
               "loss_disc_target": 0.0, "loss_disc_source": 0.0, "loss_disc_total": 0.0}
        g_correct, g_total = 0, 0
        best_mIoU = 0.0
        max_iter = epochs * iterations
        lambda_adv = max(lambda_, (lambda_ * 10) - 0.001 * epoch)
        for i in tqdm(range(iterations), total=iterations, desc=f"Epoch {epoch}"):
            source_image, source_label = next(iter(source_dataloader))
            target_image, _ = next(iter(target_dataloader))
            source_image, source_label = source_image.to(device), source_label.to(device)
            source_label = source_label.squeeze(1)
            target_image = target_image.to(device)
            current_iter = epoch * iterations + i
            if current_iter % lr_decay_iter == 0 and current_iter <= max_iter:
                dis_lr = utils.poly_lr_scheduler(discriminator_optimizer, dis_init_lr, current_iter,
                                                 lr_decay_iter, max_iter, dis_power)
                gen_lr = utils.poly_lr_scheduler(generator_optimizer, gen_init_lr, current_iter,
                                                 lr_decay_iter, max_iter, dis_power)
            *losses, corr = da2_step(generator, discriminator, generator_optimizer,
                                     discriminator_optimizer, generator_loss, discriminator_loss,
                                     source_image, source_label, target_image, lambda_adv)
            vals = _host_values(list(losses) + [corr[0]])
            for k, v in zip(("loss_gen_source", "loss_adversarial", "loss_gen_total",
                             "loss_disc_target", "loss_disc_source", "loss_disc_total"), vals):
                run[k] += v
            g_correct += int(vals[6])
            g_total += source_label.size(0) * source_label.size(1) * source_label.size(2) * dp_world()
        print(f"Epoch Results {epoch}")
        utils.tabular_print({"Genrator Accuracy": (100.0 * g_correct / g_total),
                             "dis_lr": dis_lr if dis_lr else -1, "gen_lr": gen_lr if gen_lr else -1})
        for cb in callbacks:
            cb.on_epoch_end(epoch, {
                "dis_lr": dis_lr if dis_lr else -1, "gen_lr": gen_lr if gen_lr else -1,
                "loss_gen_source": run["loss_gen_source"] / iterations,
                "loss_adversarial": run["loss_adversarial"] / iterations,
                "loss_disc_source": run["loss_disc_source"] / iterations,
                "loss_disc_target": run["loss_disc_target"] / iterations,
                "loss_disc_total": run["loss_disc_total"] / iterations,
                "loss_gen_total": run["loss_gen_total"] / iterations,
                "Genrator Accuracy": 100.0 * g_correct / g_total})
        if do_validation != -1 and epoch % do_validation == 0 and epoch != 0:
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


__all__ = ["train", "adversarial_train", "adversarial_train_2", "seg_step", "da_step", "da2_step",
           "Callback"]
