"""CPU restatement of the reference's hot-path step bodies (TEST INFRASTRUCTURE).

* ``poly_lr``  -- utils.poly_lr_scheduler (reference utils.py:33-48)
* ``seg_step`` -- one iteration of train.train (train.py:65-113)
* ``da_step``  -- one iteration of train.adversarial_train (train.py:172-284)

They are written against plain torch modules / optimizers so the same functions drive
the oracle models; the HIP path has its own loop in ``rtsds_amd.train``.
"""
import torch
import torch.nn.functional as F


def poly_lr(optimizer, init_lr, it, max_iter, power):
    lr = init_lr * (1 - it / max_iter) ** power
    optimizer.param_groups[0]["lr"] = lr
    return lr


def seg_step(model, optimizer, criterion, x, y):
    """train.py:74-106: zero_grad, fwd, sum of CE over (main, aux1, aux2), backward, step."""
    optimizer.zero_grad()
    outs = model(x)
    main, a1, a2 = outs if isinstance(outs, tuple) else (outs, None, None)
    loss = criterion(main, y)
    for a in (a1, a2):
        if a is not None:
            loss = loss + criterion(a, y)
    loss.backward()
    optimizer.step()
    correct = int(main.argmax(1).eq(y).sum())
    return {"loss": float(loss), "correct": correct, "total": y.numel()}


def da_step(G, D, optG, optD, ce, bce, src, lbl, tgt, lambda_, iterations):
    """train.py:174-275 (one inner iteration; LR scheduling is the caller's)."""
    optG.zero_grad()
    optD.zero_grad()
    for p in D.parameters():
        p.requires_grad_(False)
    out = G(src)
    if isinstance(out, tuple):
        l_seg = ce(out[0], lbl)
        for a in out[1:]:
            if a is not None:
                l_seg = l_seg + ce(a, lbl)
        src_feat = out[0]
    else:
        l_seg, src_feat = ce(out, lbl), out
    l_seg = l_seg / iterations
    l_seg.backward()

    tout = G(tgt)
    tgt_feat = tout[0] if isinstance(tout, tuple) else tout
    pred = D(F.softmax(tgt_feat, dim=1))
    l_adv = lambda_ * bce(pred, torch.ones_like(pred)) / iterations
    l_adv.backward()

    for p in D.parameters():
        p.requires_grad_(True)
    src_feat, tgt_feat = src_feat.detach(), tgt_feat.detach()
    ps = D(F.softmax(src_feat, dim=1))
    l_ds = bce(ps, torch.ones_like(ps)) / iterations
    l_ds.backward()
    pt = D(F.softmax(tgt_feat, dim=1))
    l_dt = bce(pt, torch.zeros_like(pt)) / iterations
    l_dt.backward()

    optG.step()
    optD.step()
    correct = int(src_feat.argmax(1).eq(lbl).sum())
    return {"loss_gen_source": float(l_seg), "loss_adversarial": float(l_adv),
            "loss_disc_source": float(l_ds), "loss_disc_target": float(l_dt),
            "correct": correct, "total": lbl.numel()}
