"""Deterministic per-key weight recipe (TEST INFRASTRUCTURE; mirrored by rtsds_amd.utils).

Reference weights are random-init / ImageNet downloads (build_contextpath.py:8,35,
deeplabv2.py:180-188), neither reproducible offline.  Every parity test therefore loads
the SAME synthetic ``state_dict`` into the reference (golden generation), the oracle and
the HIP path: each tensor is drawn from ``np.random.default_rng([seed, crc32(key)])`` so
the value depends only on (seed, key, shape), never on iteration order.

* conv / linear weight (ndim >= 2): N(0, 1) * sqrt(2 / fan_in)   (kaiming fan_in, as
  build_bisenet.py:130-139 does for the non-context-path convs)
* BN weight: 1 + 0.1 N(0,1); BN bias / conv bias: 0.1 N(0,1)
* running_mean: 0.1 N(0,1); running_var: U(0.5, 1.5); num_batches_tracked: 0
"""
import zlib

import numpy as np
import torch


def _rng(seed, key):
    return np.random.default_rng([int(seed), zlib.crc32(key.encode())])


def recipe_tensor(key, shape, seed, is_bn_param):
    rng = _rng(seed, key)
    shape = tuple(shape)
    if key.endswith("num_batches_tracked"):
        return np.zeros(shape, np.int64)
    if key.endswith("running_mean"):
        return (0.1 * rng.standard_normal(shape)).astype(np.float32)
    if key.endswith("running_var"):
        return rng.uniform(0.5, 1.5, shape).astype(np.float32)
    if len(shape) >= 2:
        fan_in = int(np.prod(shape[1:]))
        return (rng.standard_normal(shape) * np.sqrt(2.0 / fan_in)).astype(np.float32)
    if is_bn_param and key.endswith("weight"):
        return (1.0 + 0.1 * rng.standard_normal(shape)).astype(np.float32)
    return (0.1 * rng.standard_normal(shape)).astype(np.float32)


def recipe_state_dict(state_dict_shapes, seed=0):
    """``state_dict_shapes``: ordered mapping key -> shape.  Returns key -> torch tensor."""
    keys = list(state_dict_shapes)
    bn_prefixes = {k[: -len("running_mean")] for k in keys if k.endswith("running_mean")}
    out = {}
    for k, shp in state_dict_shapes.items():
        prefix = k.rsplit(".", 1)[0] + "."
        out[k] = torch.from_numpy(recipe_tensor(k, shp, seed, prefix in bn_prefixes))
    return out


def apply_recipe(model, seed=0):
    sd = model.state_dict()
    new = recipe_state_dict({k: tuple(v.shape) for k, v in sd.items()}, seed)
    model.load_state_dict(new)
    return model


def synthetic_images(n, h, w, seed):
    """ImageNet-normalised 0-255 images, the reference's real input distribution
    (read_image(...).float() then Normalize, datasets/cityscapes.py:62, main.py:69-72)."""
    g = torch.Generator().manual_seed(seed)
    x = torch.randint(0, 256, (n, 3, h, w), generator=g).float()
    mean = torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)
    std = torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)
    return (x - mean) / std


def synthetic_labels(n, h, w, seed, num_classes=19):
    """Labels in [0, num_classes] with num_classes == ignore (main.py:76, utils.py:67-75)."""
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, num_classes + 1, (n, h, w), generator=g)
