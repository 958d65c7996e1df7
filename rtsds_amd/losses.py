"""Loss modules on the HIP kernels: drop-ins for the nn.CrossEntropyLoss(ignore_index) and
nn.BCEWithLogitsLoss() built by the reference's optimzer_loss_loader (main.py:124-134)."""
import torch
from torch import nn

from . import functional as F
from .runtime import dp_world


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
    """Mean of the logistic loss.  Under data parallelism the mean runs over every rank's
    elements: every eager call all-reduces the local element count (a one-element collective,
    issued by every rank on every call, so the collectives of the ranks always pair up) and
    scales this rank's mean by n / total on the device (no host sync).  Under hipGraph capture
    (runtime.GraphedStep) no collective may run inside the captured segment, so the call reuses
    the scale of the last eager call with the same local size (the warm-up iterations before
    capture); graph replays have static shapes, so that scale stays valid.  A capture that meets
    a local size no eager call has seen raises instead of guessing."""

    def __init__(self, reduction="mean"):
        super().__init__()
        if reduction != "mean":
            raise NotImplementedError("rtsds_amd.BCEWithLogitsLoss: mean only (main.py:132)")
        self._scale = {}

    def forward(self, input, target):
        loss = F.bce_with_logits(input, target)
        if dp_world() == 1:
            return loss
        # global-batch mean under data parallelism (see runtime.dp_world): this rank's mean
        # weighted by its share of the all-reduced element count, so shards of unequal size
        # still sum to the gathered-batch mean
        import torch.distributed as dist
        n = int(input.numel())
        key = (n, dp_world())
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            scale = self._scale.get(key)
            if scale is None:
                raise RuntimeError("rtsds_amd.BCEWithLogitsLoss: run an eager iteration with this local "
                                   "batch size before graph capture")
            return loss * scale
        cnt = torch.full((1,), float(n), dtype=torch.float64, device=input.device)
        dist.all_reduce(cnt)
        # fp32(n / total): the rounding ATen applies to a Python-float multiplier
        scale = (n / cnt).to(loss.dtype).reshape(())
        self._scale[key] = scale
        return loss * scale
