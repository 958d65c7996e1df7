"""Device-side input pipeline: the reference's torchvision transforms (main.py:25-108) as HIP
kernels (csrc/data.hip) over decoded uint8 HWC images in HBM.

Reference pipelines (main.py:60-96), reproduced here per sample of a batch:

* Cityscapes image:  Resize(image_size, antialias=True) -> Normalize(mean, std)
* Cityscapes label:  Resize(image_size, antialias=True) -> IntRangeTransformer(0, num_classes)
* GTA5 image:        [RandomApply([GaussianBlur(k, sigma), RandomHorizontalFlip(p)], p)] ->
                     Resize(image_size) -> Normalize(mean, std)
* GTA5 label:        Resize(image_size)   (the augmentation flips the image only, as the
                     reference's pipeline does)

The image comes out in the network's input layout (NHWC, the runtime compute dtype), so the
model's input packing is a no-op; labels come out int64 [N, 1, H, W] as the reference's loaders
deliver them (train.py squeezes dim 1).  Random decisions draw from torch's CPU generator in
torchvision's call order (RandomApply's coin, GaussianBlur's sigma, the flip coin).
"""
import torch

from ._lib import lib
from .runtime import CL, compute_dtype, stream, workspace

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def _check(code, what):
    if code != 0:
        raise RuntimeError(f"rtsds_amd.transforms: {what} failed (status {code})")


class GaussianBlur:
    """torchvision GaussianBlur(kernel_size, sigma): sigma ~ U(sigma_min, sigma_max) per call."""

    def __init__(self, kernel_size, sigma=(0.1, 2.0)):
        ks = (kernel_size, kernel_size) if isinstance(kernel_size, int) else tuple(kernel_size)
        if any(k <= 0 or k % 2 == 0 for k in ks):
            raise ValueError("Kernel size value should be an odd and positive number.")
        self.kernel_size = ks
        self.sigma = (sigma, sigma) if isinstance(sigma, (int, float)) else tuple(sigma)

    def params(self):
        return float(torch.empty(1).uniform_(self.sigma[0], self.sigma[1]).item())


class RandomHorizontalFlip:
    def __init__(self, p=0.5):
        self.p = p


class RandomApply:
    """RandomApply(transforms, p): the listed transforms all run with probability p."""

    def __init__(self, transforms, p=0.5):
        self.transforms = list(transforms)
        self.p = p


def augmentation_loader(config, probability):
    """main.py:46-58 / 25-44: RandomApply over the configured augmentations."""
    aug = config.augmentation
    out = []
    for key in aug.keys():
        if key == "GaussianBlur":
            c = aug["GaussianBlur"]
            out.append(GaussianBlur(kernel_size=[int(i) for i in str(c["kernel_size"]).split(",")],
                                    sigma=[float(i) for i in str(c["sigma"]).split(",")]))
        elif key == "RandomHorizontalFlip":
            out.append(RandomHorizontalFlip(p=aug["RandomHorizontalFlip"]["p"]))
        elif key in ("ColorJitter", "ColorJitterWithRandomBrightness"):
            raise NotImplementedError("rtsds_amd.transforms: ColorJitter is not implemented (the reference "
                                      "config has it commented out, config.yaml:111-123)")
    return RandomApply(out, p=probability)


def _decisions(augment):
    """(blur sigma or None, flip) for one sample, drawing in torchvision's order."""
    if augment is None or not augment.transforms:
        return None, False
    if augment.p < torch.rand(1):
        return None, False
    sigma, flip = None, False
    for t in augment.transforms:
        if isinstance(t, GaussianBlur):
            sigma = (t, t.params())
        elif isinstance(t, RandomHorizontalFlip):
            flip = bool(torch.rand(1) < t.p)
    return sigma, flip


def _as_hwc_u8(img):
    if img.dtype != torch.uint8:
        raise RuntimeError("rtsds_amd.transforms: decoded uint8 images expected")
    if img.dim() == 2:
        img = img.unsqueeze(-1)
    return img.contiguous()


class ImagePipeline:
    """Resize(size, antialias=True) [after the optional augmentation] -> Normalize, into slot n
    of an NHWC batch in the compute dtype."""

    def __init__(self, size, mean=IMAGENET_MEAN, std=IMAGENET_STD, augment=None):
        self.size = (int(size[0]), int(size[1]))
        self.mean, self.std = tuple(mean), tuple(std)
        self.augment = augment
        self._ms = {}

    def _mean_std(self, device):
        if device not in self._ms:
            t = torch.tensor(list(self.mean) + list(self.std), dtype=torch.float32).to(device)
            self._ms[device] = (t, t[3:])
        return self._ms[device]

    def __call__(self, images, dtype=None):
        """images: list of uint8 HWC [H_i, W_i, 3] device tensors -> [N, 3, Ho, Wo] NHWC."""
        dtype = dtype or compute_dtype()
        dev = images[0].device
        ho, wo = self.size
        out = torch.empty((len(images), 3, ho, wo), dtype=dtype, device=dev, memory_format=CL)
        ms, sd = self._mean_std(dev)
        for n, img in enumerate(images):
            img = _as_hwc_u8(img)
            h, w, c = img.shape
            src, src_u8 = img, 1
            sigma, flip = _decisions(self.augment)
            if sigma is not None:
                blur, s = sigma
                src = torch.empty((h, w, c), dtype=torch.float32, device=dev)
                _check(lib.rtsds_gaussian_blur(img.data_ptr(), 1, src.data_ptr(), c, h, w, blur.kernel_size[0],
                                               blur.kernel_size[1], s, s, stream()), "gaussian blur")
                src_u8 = 0
            ws = workspace(lib.rtsds_resize_aa_workspace(c, h, w, ho, wo), dev)
            dst = out[n].permute(1, 2, 0)  # this image's HWC slot of the NHWC batch
            _check(lib.rtsds_resize_aa(src.data_ptr(), src_u8, c, h, w, dst.data_ptr(),
                                       1 if dtype == torch.bfloat16 else 0, ho, wo, int(flip), ms.data_ptr(),
                                       sd.data_ptr(), 0, -1, ws.data_ptr(), ws.numel(), stream()), "resize")
        return out


class LabelPipeline:
    """Resize(size, antialias=True) of an id map (interpolated in float, rounded half-to-even)
    -> optional IntRangeTransformer(lo, hi) clamp; int64 [N, 1, Ho, Wo]."""

    def __init__(self, size, clamp=None):
        self.size = (int(size[0]), int(size[1]))
        self.clamp = clamp

    def __call__(self, labels):
        dev = labels[0].device
        ho, wo = self.size
        out = torch.empty((len(labels), 1, ho, wo), dtype=torch.int64, device=dev)
        lo, hi = self.clamp if self.clamp is not None else (0, -1)
        for n, lab in enumerate(labels):
            lab = _as_hwc_u8(lab) if lab.dtype == torch.uint8 else lab
            if lab.dtype == torch.int64:  # decoded GTA5 ids: interpolate from a float copy
                src, u8 = lab.reshape(lab.shape[-2], lab.shape[-1], 1).float().contiguous(), 0
            else:
                src, u8 = lab, 1
            h, w = src.shape[0], src.shape[1]
            ws = workspace(lib.rtsds_resize_aa_workspace(1, h, w, ho, wo), dev)
            _check(lib.rtsds_resize_aa(src.data_ptr(), u8, 1, h, w, out[n].data_ptr(), 2, ho, wo, 0, None, None,
                                       int(lo), int(hi), ws.data_ptr(), ws.numel(), stream()), "label resize")
        return out


def decode_gta5_labels(rgb):
    """GTA5 RGB colour label (uint8 HWC, device) -> train ids int64 [H, W] (gta5.py:111-118)."""
    rgb = _as_hwc_u8(rgb)
    h, w = rgb.shape[0], rgb.shape[1]
    out = torch.empty((h, w), dtype=torch.int64, device=rgb.device)
    _check(lib.rtsds_gta5_decode(rgb.data_ptr(), out.data_ptr(), h, w, stream()), "gta5 decode")
    return out


def collate_raw(batch):
    """DataLoader collate for raw samples of different sizes: lists of uint8 tensors."""
    return [b[0] for b in batch], [b[1] for b in batch]


class DeviceLoader:
    """A DataLoader of raw samples -> batches ready for the network: images moved to the device
    (pinned, non-blocking) and run through ``image_pipe``, labels through ``label_pipe`` (GTA5
    colour labels decoded first when ``decode_rgb_labels``).  Same iteration / len semantics as
    the wrapped loader, so train.train / adversarial_train consume it unchanged."""

    def __init__(self, loader, image_pipe, label_pipe, device="cuda", decode_rgb_labels=False):
        self.loader = loader
        self.image_pipe, self.label_pipe = image_pipe, label_pipe
        self.device = device
        self.decode = decode_rgb_labels
        self.epoch = 0

    def __len__(self):
        return len(self.loader)

    def _move(self, ts):
        if torch.device(self.device).type == "cpu":
            return list(ts)
        return [t.pin_memory().to(self.device, non_blocking=True) if t.device.type == "cpu" else t for t in ts]

    def __iter__(self):
        # A DistributedSampler replays the permutation of its current epoch on every iter();
        # the reference's RandomSampler draws a new one each time (adversarial_train takes
        # next(iter(loader)) per iteration, train.py:186-187), so every new iterator advances
        # the sampler's epoch.
        sampler = getattr(self.loader, "sampler", None)
        if hasattr(sampler, "set_epoch"):
            sampler.set_epoch(self.epoch)
            self.epoch += 1
        for images, labels in self.loader:
            images, labels = self._move(images), self._move(labels)
            if self.decode:
                labels = [decode_gta5_labels(t) for t in labels]
            yield self.image_pipe(images), self.label_pipe(labels)


def parse_size(s):
    return [int(v) for v in str(s).split(",")]


__all__ = ["ImagePipeline", "LabelPipeline", "DeviceLoader", "GaussianBlur", "RandomHorizontalFlip", "RandomApply",
           "augmentation_loader", "decode_gta5_labels", "collate_raw", "parse_size"]
