"""Validation loops (reference validation.py:12-148) with the argmax and the 19x19 confusion
histogram computed on the device (rtsds_argmax + rtsds_confusion); mIoU is
``utils.per_class_iou`` over the accumulated histogram exactly as the reference computes it.

Deviation (documented): ``val`` also accepts ``class_names`` / ``detailed_report`` -- the
reference's main.py:365-374 passes them and its ``val`` raises TypeError.
"""
import numpy as np
import torch

from . import functional as F
from . import utils


def _confusion_device(model, val_loader, num_classes, device, callbacks):
    hist = torch.zeros(num_classes * num_classes, dtype=torch.int64, device=device)
    for batch_idx, (inputs, targets) in enumerate(val_loader):
        inputs = inputs.to(device)
        targets = targets.to(device)
        if targets.dim() == 4:
            targets = targets.squeeze(1)
        outputs = model(inputs)
        if isinstance(outputs, tuple):
            outputs = outputs[0]
        pred = F.argmax_channels(outputs)
        F.confusion(targets.long(), pred, hist, num_classes)
        if callbacks:
            h = hist.view(num_classes, num_classes).cpu().numpy()
            tp = np.diag(h)
            loss = 1.0 - np.sum(tp) / max(np.sum(h), 1)
            for cb in callbacks:
                cb.on_validation_batch_end(batch_idx, loss)
    return hist.view(num_classes, num_classes).cpu().numpy()


def val(epoch, model, val_loader, num_classes, device="cuda", callbacks=[], class_names=None,
        detailed_report=False):
    for cb in callbacks:
        cb.on_validation_begin()
    model.eval()
    with torch.no_grad():
        hist = _confusion_device(model, val_loader, num_classes, device, callbacks)
    ious = utils.per_class_iou(hist)
    mean_iou = np.nanmean(ious)
    print(f"Validation Mean IoU for Epoch {epoch + 1}: {mean_iou:.4f}")
    for cb in callbacks:
        cb.on_validation_end(mean_iou)
    return mean_iou


def val_GTA5(epoch, model, val_loader, num_classes, class_names, callbacks=[], device="cuda"):
    import pandas as pd
    model.eval()
    for cb in callbacks:
        cb.on_validation_begin()
    with torch.no_grad():
        hist = _confusion_device(model, val_loader, num_classes, device, callbacks)
    ious = utils.per_class_iou(hist)
    total_miou = np.nanmean(ious)
    print(f"Validation mIoU for Epoch {epoch + 1}: {total_miou:.4f}")
    df = pd.DataFrame({"Class": class_names, "IoU": [f"{i:.4f}" for i in ious]})
    print(df)
    for cb in callbacks:
        cb.on_validation_end({"validation_mIoU": total_miou}, data=df)
    return total_miou, df
