"""CPU restatement of the reference's hot-path step bodies (TEST INFRASTRUCTURE).

* ``poly_lr``  -- utils.poly_lr_scheduler (reference utils.py:33-48)
* ``seg_step`` -- one iteration of train.train (train.py:65-113)
* ``da_step``  -- one iteration of train.adversarial_train (train.py:172-284)
* ``da2_step`` -- one iteration of train.adversarial_train_2 (train.py:373-466)

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
    return {"loss_gen_source": float(l_seg.detach()), "loss_adversarial": float(l_adv.detach()),
            "loss_disc_source": float(l_ds.detach()), "loss_disc_target": float(l_dt.detach()),
            "correct": correct, "total": lbl.numel()}


def da2_step(G, D, optG, optD, ce, bce, src, lbl, tgt, lambda_adv):
    """train.py:373-466 (one inner iteration; LR scheduling is the caller's)."""
    th, tw = tgt.shape[2], tgt.shape[3]
    real = torch.ones(tgt.shape[0], 1, 1, 1)
    fake = torch.zeros(tgt.shape[0], 1, 1, 1)
    optG.zero_grad()
    out = G(src)
    if isinstance(out, tuple):
        l_seg = ce(out[0], lbl)
        for a in out[1:]:
            if a is not None:
                l_seg = l_seg + ce(a, lbl)
        out = out[0]
    else:
        l_seg = ce(out, lbl)
    correct = int(out.argmax(1).eq(lbl).sum())
    t = G(tgt)
    t = t[0] if isinstance(t, tuple) else t
    t = F.adaptive_avg_pool2d(t, (th, tw))
    l_adv = bce(D(F.softmax(t, dim=1)), fake)
    g_loss = l_seg + lambda_adv * l_adv
    g_loss.backward()
    optG.step()
    optD.zero_grad()
    with torch.no_grad():
        fs = G(src)
        fs = F.adaptive_avg_pool2d(fs[0] if isinstance(fs, tuple) else fs, (th, tw))
        rs = G(tgt)
        rs = F.adaptive_avg_pool2d(rs[0] if isinstance(rs, tuple) else rs, (th, tw))
    d_real = bce(D(F.softmax(rs, dim=1)), real)
    d_fake = bce(D(F.softmax(fs, dim=1)), fake)
    d_loss = d_real + d_fake
    d_loss.backward()
    optD.step()
    return {"loss_gen_source": float(l_seg), "loss_adversarial": float(l_adv),
            "loss_gen_total": float(g_loss), "loss_disc_target": float(d_real),
            "loss_disc_source": float(d_fake), "loss_disc_total": float(d_loss),
            "correct": correct, "total": lbl.numel()}
