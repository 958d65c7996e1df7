"""Host-side helpers of the hot path (reference utils.py).

* ``poly_lr_scheduler``  -- utils.py:33-48 (same formula, writes param_groups[0]['lr'])
* ``forModel``           -- utils.py:97-107.  The reference wraps >1 GPU in nn.DataParallel
  (single process, GPU0 master).  Here data parallelism is one process per GPU: when
  launched by torchrun (WORLD_SIZE > 1) the RCCL process group is initialised and the model is
  placed on LOCAL_RANK's device; rtsds_amd.optim.Adam all-reduces the flat gradients.
* ``fast_hist`` / ``per_class_iou`` -- utils.py:52-63 (numpy, used by validation)
* ``IntRangeTransformer`` / ``tabular_print`` -- utils.py:67-94 (the no-prettytable fallback
  prints the DataFrame; the reference's references an unimported ``sys``)
"""
import os

import numpy as np
import torch


def poly_lr_scheduler(optimizer, init_lr, iter, lr_decay_iter=1, max_iter=300, power=0.9):
    lr = init_lr * (1 - iter / max_iter) ** power
    optimizer.param_groups[0]["lr"] = lr
    return lr


def fast_hist(a, b, n):
    k = (a >= 0) & (a < n)
    return np.bincount(n * a[k].astype(int) + b[k], minlength=n ** 2).reshape(n, n)


def per_class_iou(hist):
    epsilon = 1e-5
    return (np.diag(hist)) / (hist.sum(1) + hist.sum(0) - np.diag(hist) + epsilon)


class IntRangeTransformer:
    def __init__(self, min_val=0, max_val=255):
        self.min_val, self.max_val = min_val, max_val

    def __call__(self, sample):
        return torch.clamp(sample, self.min_val, self.max_val).long()


def tabular_print(log_dict):
    import pandas as pd
    df = pd.DataFrame({**log_dict}, index=[0])
    try:
        from prettytable import PrettyTable
    except ImportError:
        print(df)
        return
    x = PrettyTable()
    for col in df.columns:
        x.add_column(col, df[col].values)
    print(x)


def dist_env():
    """(rank, local_rank, world) from torchrun's environment (1 process per GPU)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return rank, local, world


def init_distributed(backend=None):
    """Initialise torch.distributed from the torchrun environment (no-op for world 1).
    backend: 'nccl' (= RCCL over xGMI on ROCm) for HIP tensors, 'gloo' for CPU tests."""
    import torch.distributed as dist
    rank, local, world = dist_env()
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return rank, local, world


def forModel(model, device):
    rank, local, world = dist_env()
    if device == "cuda":
        if world > 1:
            init_distributed("nccl")
            model = model.to(torch.device("cuda", local))
        else:
            model = model.cuda()
        if rank == 0:
            print("The number of cuda GPUs : ", torch.cuda.device_count(), "(processes:", world, ")")
    return model


def count_parameters(model):
    return sum(p.numel() for p in model.parameters() if p.requires_grad)
