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
    elements.  D's logits have a data-independent size, so the global element count is
    all-reduced once per local size and cached.  The cache miss is a collective, so every rank
    must miss on the same calls: each rank's sequence of local sizes must be fixed from the
    first iteration on -- equal shards (DistributedSampler pads its shards to equal length,
    synthetic loaders are equal, main.py's loaders drop_last) or unequal but fixed shards
    (those get the exact weighted mean).  A rank that meets a new local size while another
    rank hits its cache would desynchronise the collectives, and that case is NOT detected: the
    check on a miss (every rank taking part, equal cache lengths) only catches ranks that miss
    together with different cache histories.  The missing rank's count all-reduce would pair
    with the other rank's next collective."""

    def __init__(self, reduction="mean"):
        super().__init__()
        if reduction != "mean":
            raise NotImplementedError("rtsds_amd.BCEWithLogitsLoss: mean only (main.py:132)")
        self._global = {}

    def forward(self, input, target):
        loss = F.bce_with_logits(input, target)
        if dp_world() == 1:
            return loss
        # global-batch mean under data parallelism (see runtime.dp_world): this rank's mean
        # weighted by its share of the all-reduced element count, so shards of unequal size
        # still sum to the gathered-batch mean (a graph-segment break under capture)
        import torch.distributed as dist
        n = int(input.numel())
        total = self._global.get((n, dp_world()))
        if total is None:
            if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
                raise RuntimeError("rtsds_amd.BCEWithLogitsLoss: run an eager iteration before graph capture")
            # [local count, 1, number of cached sizes]: the second slot counts the ranks taking
            # part, the third must agree (all ranks miss together on the same call)
            cnt = torch.tensor([float(n), 1.0, float(len(self._global))], dtype=torch.float64, device=input.device)
            dist.all_reduce(cnt)  # eager, outside any graph capture: warm-up iterations fill the cache
            w = dist.get_world_size()  # the ranks the collective actually ran over
            if int(cnt[1].item()) != w or float(cnt[2].item()) != w * len(self._global):
                raise RuntimeError("rtsds_amd.BCEWithLogitsLoss: ranks disagree on the global element count "
                                   "cache (local batch sizes must follow the same pattern on every rank)")
            total = self._global[(n, dp_world())] = float(cnt[0].item())
        return loss * (n / total)
