"""rtsds_amd -- MI355X-native (gfx950 / CDNA4) implementation of the RTSDS hot path.

BiSeNet / DeepLabV2 forward+backward and the adversarial domain-adaptation discriminator
step of sina-behnam/RTSDS (train.py), behind the reference's module / loop / config API.
Compute runs only in librtsds_hip.so (hand-written HIP kernels, C ABI in
include/rtsds_hip.h); PyTorch supplies device memory, streams, autograd plumbing and
torch.distributed (RCCL).
"""
from .runtime import compute_dtype, precision, set_compute_dtype  # noqa: F401

__all__ = ["compute_dtype", "precision", "set_compute_dtype"]
