"""CPU restatement of the reference's input transforms (TEST INFRASTRUCTURE).

The reference builds them from torchvision 0.18 (main.py:25-96), which is not installed here;
this restates the torchvision semantics the pipeline relies on with plain torch ops:

* Resize(size[, antialias=True]) on a tensor: float images go through
  F.interpolate(mode="bilinear", align_corners=False, antialias=True); integer tensors are
  cast to float32, interpolated, rounded (torch.round: half to even) and cast back
  (torchvision transforms/_functional_tensor.py resize / _cast_squeeze_in / _cast_squeeze_out).
* Normalize(mean, std): (x - mean[c]) / std[c].
* RandomHorizontalFlip: x.flip(-1).
* GaussianBlur(kernel_size, sigma): 1-D kernels pdf = exp(-0.5 (x / sigma)^2) over
  x = linspace(-(k-1)/2, (k-1)/2, k), normalised; 2-D kernel = ky^T kx; reflect pad k // 2;
  depthwise conv2d (_functional_tensor.py gaussian_blur, _get_gaussian_kernel1d/2d).
* IntRangeTransformer(lo, hi): clamp().long() (reference utils.py:67-75).
* GTA5 RGB label decode: gta5.py:111-118's loop over train ids (later ids overwrite).
Parity is unpinned by reference fixtures (torchvision absent; the reference has no tests):
it rests on torch's own interpolate / conv2d and the cited torchvision source semantics.
"""
import torch
import torch.nn.functional as F

TRAIN_ID_COLORS = [
    (128, 64, 128), (244, 35, 232), (70, 70, 70), (102, 102, 156), (190, 153, 153), (153, 153, 153),
    (250, 170, 30), (220, 220, 0), (107, 142, 35), (152, 251, 152), (70, 130, 180), (220, 20, 60),
    (255, 0, 0), (0, 0, 142), (0, 0, 70), (0, 60, 100), (0, 80, 100), (0, 0, 230), (119, 11, 32)]


def resize(img, size, antialias=True):
    """img [..., C, H, W] (float or integer)."""
    out_dtype = img.dtype
    x = img.float() if not img.dtype.is_floating_point else img
    squeeze = x.dim() == 3
    if squeeze:
        x = x.unsqueeze(0)
    y = F.interpolate(x, size=list(size), mode="bilinear", align_corners=False, antialias=antialias)
    if squeeze:
        y = y.squeeze(0)
    if not out_dtype.is_floating_point:
        y = torch.round(y).to(out_dtype)
    return y


def normalize(x, mean, std):
    m = torch.tensor(mean, dtype=x.dtype).view(-1, 1, 1)
    s = torch.tensor(std, dtype=x.dtype).view(-1, 1, 1)
    return (x - m) / s


def _gauss1d(k, sigma):
    half = (k - 1) * 0.5
    x = torch.linspace(-half, half, steps=k)
    pdf = torch.exp(-0.5 * (x / sigma).pow(2))
    return pdf / pdf.sum()


def gaussian_blur(img, kernel_size, sigma):
    """img float [C, H, W]; kernel_size (kx, ky); sigma (sx, sy)."""
    kx, ky = kernel_size
    k2 = torch.mm(_gauss1d(ky, sigma[1])[:, None], _gauss1d(kx, sigma[0])[None, :])
    c = img.shape[0]
    w = k2.expand(c, 1, ky, kx)
    x = F.pad(img.unsqueeze(0), [kx // 2, kx // 2, ky // 2, ky // 2], mode="reflect")
    return F.conv2d(x, w, groups=c).squeeze(0)


def int_range(x, lo, hi):
    return torch.clamp(x, lo, hi).long()


def decode_gta5(rgb_chw):
    """[3, H, W] int -> [H, W] long (gta5.py:111-118)."""
    out = torch.zeros(rgb_chw.shape[1:], dtype=torch.long)
    for i, c in enumerate(TRAIN_ID_COLORS):
        mask = torch.all(rgb_chw == torch.tensor(c).view(3, 1, 1), dim=0)
        out[mask] = i
    return out
