"""Loss modules on the HIP kernels: drop-ins for the nn.CrossEntropyLoss(ignore_index) and
nn.BCEWithLogitsLoss() built by the reference's optimzer_loss_loader (main.py:124-134)."""
import torch
from torch import nn

from . import functional as F
from .runtime import collective, dp_world


class CrossEntropyLoss(nn.Module):
    """Mean over non-ignored pixels of -log softmax(x)[target]; logits [N, C, H, W] (NHWC or
    NCHW memory), target int64 [N, H, W] (or [N, 1, H, W]).  Under data parallelism the mean
    runs over every rank's pixels (runtime.dp_world)."""

    def __init__(self, weight=None, ignore_index=-100, reduction="mean"):
        super().__init__()
        if weight is not None or reduction != "mean":
            raise NotImplementedError("rtsds_amd.CrossEntropyLoss: unweighted mean only (main.py:130)")
        self.ignore_index = -100 if ignore_index is None else int(ignore_index)

    def forward(self, input, target):
        return F.cross_entropy(input, target, self.ignore_index)


class BCEWithLogitsLoss(nn.Module):
    def __init__(self, reduction="mean"):
        super().__init__()
        if reduction != "mean":
            raise NotImplementedError("rtsds_amd.BCEWithLogitsLoss: mean only (main.py:132)")

    def forward(self, input, target):
        loss = F.bce_with_logits(input, target)
        if dp_world() == 1:
            return loss
        # global-batch mean under data parallelism (see runtime.dp_world): this rank's mean
        # weighted by its share of the all-reduced element count, so shards of unequal size
        # still sum to the gathered-batch mean (a graph-segment break under capture)
        import torch.distributed as dist
        n = float(input.numel())
        cnt = torch.full((1,), n, dtype=torch.float32, device=input.device)
        collective(lambda: dist.all_reduce(cnt))
        return loss * (n / cnt[0])
