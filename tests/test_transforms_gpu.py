"""Device input pipeline (rtsds_amd.transforms, csrc/data.hip) vs the CPU restatement of the
reference's torchvision transforms (oracle/transforms.py).  The resize / normalize / blur
arithmetic is torchvision's: parity unpinned by reference fixtures (torchvision is absent and
the reference has no tests); the checker is torch's own interpolate / conv2d on the CPU.  The
GTA5 colour decode and the IntRangeTransformer clamp are the reference's own code and are
pinned by fixtures captured from it (tests/golden/inputs.npz, tests/test_inputs_golden.py).

Tolerances: images in fp32 -- |err| <= 2e-5 x max|ref| (the same separable weights; fma vs
separate multiply-add in the taps); bf16 images -- the fp32 result rounded once (2^-8 rel);
labels (integers from a float interpolation rounded half-to-even) -- identical except at most
1e-4 of the pixels within 1 of the reference (ties rounding the other way).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)

from oracle import transforms as OT  # noqa: E402
from rtsds_amd import transforms as T  # noqa: E402

DEV = "cuda"
MEAN, STD = T.IMAGENET_MEAN, T.IMAGENET_STD


def _img(h, w, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, 256, (h, w, 3), generator=g, dtype=torch.uint8)


@pytest.mark.parametrize("src,dst", [((1024, 2048), (512, 1024)),     # Cityscapes
                                     ((1052, 1914), (720, 1280)),     # GTA5 (non-integer scale)
                                     ((37, 53), (64, 96)),            # upscaling (support 1)
                                     ((100, 300), (33, 70))])         # odd downscale
@pytest.mark.parametrize("flip", [0, 1])
def test_image_resize_normalize(src, dst, flip):
    img = _img(*src, seed=src[0] + flip)
    ref = OT.normalize(OT.resize(img.permute(2, 0, 1).float(), dst), MEAN, STD)
    if flip:
        ref = OT.normalize(OT.resize(img.permute(2, 0, 1).float().flip(-1), dst), MEAN, STD)
    pipe = T.ImagePipeline(dst)
    if flip:
        pipe.augment = T.RandomApply([T.RandomHorizontalFlip(p=1.0)], p=1.0)
    out = pipe([img.to(DEV)], dtype=torch.float32)
    torch.cuda.synchronize()
    got = out[0].cpu()
    err = (got - ref).abs().max().item()
    assert err <= 2e-5 * ref.abs().max().item(), err
    out16 = pipe([img.to(DEV)], dtype=torch.bfloat16)[0].float().cpu()
    assert torch.equal(out16, got.to(torch.bfloat16).float()) or \
        ((out16 - ref).abs() <= 8e-3 * ref.abs() + 1e-2).all()


@pytest.mark.parametrize("clamp", [None, (0, 19)])
def test_label_resize_round_clamp(clamp):
    g = torch.Generator().manual_seed(3)
    lab = torch.randint(0, 20, (1024, 2048), generator=g, dtype=torch.uint8)
    lab[:100, :100] = 255  # ignore region (clamped to 19 by IntRangeTransformer)
    ref = OT.resize(lab.long().unsqueeze(0), (512, 1024)).squeeze(0)
    if clamp:
        ref = OT.int_range(ref, *clamp)
    got = T.LabelPipeline((512, 1024), clamp=clamp)([lab.to(DEV)])[0, 0].cpu()
    diff = (got != ref)
    assert diff.float().mean().item() <= 1e-4, diff.float().mean().item()
    assert (got - ref).abs().max().item() <= 1


def test_gaussian_blur_then_flip_then_resize():
    """GTA5 augmentation order (main.py:86-89): blur, flip, resize, normalize."""
    img = _img(120, 200, seed=9)
    blur = T.GaussianBlur((5, 9), (0.1, 5.0))
    torch.manual_seed(123)
    pipe = T.ImagePipeline((60, 100), augment=T.RandomApply([blur, T.RandomHorizontalFlip(1.0)], p=1.0))
    out = pipe([img.to(DEV)], dtype=torch.float32)[0].cpu()
    torch.manual_seed(123)
    torch.rand(1)  # RandomApply's coin
    sigma = torch.empty(1).uniform_(0.1, 5.0).item()
    x = OT.gaussian_blur(img.permute(2, 0, 1).float(), (5, 9), (sigma, sigma)).flip(-1)
    ref = OT.normalize(OT.resize(x, (60, 100)), MEAN, STD)
    err = (out - ref).abs().max().item()
    assert err <= 1e-4 * ref.abs().max().item(), err


def test_gta5_decode():
    g = torch.Generator().manual_seed(4)
    ids = torch.randint(0, 19, (64, 96), generator=g)
    cols = torch.tensor(OT.TRAIN_ID_COLORS, dtype=torch.uint8)
    rgb = cols[ids]  # HWC
    rgb[:5, :5] = torch.tensor([1, 2, 3], dtype=torch.uint8)  # unknown colour -> 0
    want = OT.decode_gta5(rgb.permute(2, 0, 1).long())
    got = T.decode_gta5_labels(rgb.to(DEV)).cpu()
    assert torch.equal(got, want)


def test_gta5_decode_kernel_matches_reference_fixture(golden):
    """rtsds_gta5_decode vs GTA5.__decode_label__ captured from the reference
    (tests/golden/inputs.npz: every colour of the map incl. ignore classes and shared colours,
    near-miss and random colours): identical ids."""
    arrays, _ = golden("inputs")
    rgb = torch.from_numpy(arrays["gta5_rgb"])
    want = torch.from_numpy(arrays["gta5_ids"]).long()
    got = T.decode_gta5_labels(rgb.to(DEV)).cpu()
    assert torch.equal(got, want)


def test_label_clamp_matches_reference_fixture(golden):
    """The label pipeline's IntRangeTransformer(0, 19) clamp (inside rtsds_resize_aa, at an
    identity resize so only the clamp acts) vs the reference's IntRangeTransformer captured on
    int64 labels in [-40, 300): identical."""
    arrays, _ = golden("inputs")
    x = torch.from_numpy(arrays["int_range_in_long"]).long()
    want = torch.from_numpy(arrays["int_range_out_long"]).long()
    got = T.LabelPipeline(tuple(x.shape[-2:]), clamp=(0, 19))([x.to(DEV)])[0].cpu()
    assert torch.equal(got, want)


def test_device_loader_end_to_end(tmp_path):
    """Reference-layout Cityscapes directories of PNGs -> CityScapes reader -> DataLoader ->
    DeviceLoader: NHWC compute-dtype images and int64 [N, 1, H, W] labels equal to the CPU
    restatement of the reference's transforms, and a training iteration consumes them."""
    from PIL import Image
    from torch.utils.data import DataLoader

    import rtsds_amd
    from rtsds_amd import losses, optim
    from rtsds_amd.datasets import CityScapes
    from rtsds_amd.models.bisenet.build_bisenet import BiSeNet
    from rtsds_amd.train import train
    imgs, labs = [], []
    for i in range(2):
        (tmp_path / "img" / "city").mkdir(parents=True, exist_ok=True)
        (tmp_path / "gt" / "city").mkdir(parents=True, exist_ok=True)
        a = _img(128, 256, seed=20 + i).numpy()
        l = np.random.default_rng(i).integers(0, 20, (128, 256)).astype(np.uint8)
        Image.fromarray(a).save(tmp_path / "img" / "city" / f"city_{i:06d}_000019_leftImg8bit.png")
        Image.fromarray(l).save(tmp_path / "gt" / "city" / f"city_{i:06d}_000019_gtFine_labelTrainIds.png")
        imgs.append(torch.from_numpy(a))
        labs.append(torch.from_numpy(l))
    ds = CityScapes(str(tmp_path / "gt"), str(tmp_path / "img"))
    assert len(ds) == 2
    dl = T.DeviceLoader(DataLoader(ds, batch_size=2, shuffle=False, collate_fn=T.collate_raw),
                        T.ImagePipeline((64, 128)), T.LabelPipeline((64, 128), clamp=(0, 19)))
    with rtsds_amd.precision(torch.float32):
        (x, y), = list(dl)
    assert x.is_contiguous(memory_format=torch.channels_last) and x.dtype == torch.float32
    for i in range(2):
        ref = OT.normalize(OT.resize(imgs[i].permute(2, 0, 1).float(), (64, 128)), MEAN, STD)
        assert (x[i].cpu() - ref).abs().max().item() <= 2e-5 * ref.abs().max().item()
        rl = OT.int_range(OT.resize(labs[i].long().unsqueeze(0), (64, 128)), 0, 19)
        assert (y[i].cpu() != rl).float().mean().item() <= 1e-3
    net = BiSeNet(19, "resnet18").to(DEV)
    opt = optim.Adam(net.parameters(), lr=1e-4)
    with rtsds_amd.precision(torch.bfloat16):
        train(epoch=0, model=net, train_loader=dl, criterion=losses.CrossEntropyLoss(ignore_index=19),
              optimizer=opt, init_lr=1e-4, max_iter=2, power=0.9, lr_decay_iter=1)
