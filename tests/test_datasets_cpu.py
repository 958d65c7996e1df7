"""Dataset readers on the CPU (no kernels): file discovery and id merge of the reference's
datasets/cityscapes.py:24-53 and datasets/gta5.py:50-107, PNG decode to uint8 HWC."""
import numpy as np
import pytest
import torch

PIL = pytest.importorskip("PIL")


def _png(path, arr):
    from PIL import Image
    path.parent.mkdir(parents=True, exist_ok=True)
    Image.fromarray(arr).save(path)


def test_cityscapes_discovery_and_decode(tmp_path):
    from rtsds_amd.datasets import CityScapes
    rng = np.random.default_rng(0)
    for city, n in (("aachen", 2), ("bremen", 1)):
        for i in range(n):
            stem = f"{city}_{i:06d}_000019"
            _png(tmp_path / "images" / city / f"{stem}_leftImg8bit.png", rng.integers(0, 256, (8, 16, 3), dtype=np.uint8))
            _png(tmp_path / "gtFine" / city / f"{stem}_gtFine_labelTrainIds.png", rng.integers(0, 20, (8, 16), dtype=np.uint8))
            _png(tmp_path / "gtFine" / city / f"{stem}_gtFine_color.png", rng.integers(0, 256, (8, 16, 3), dtype=np.uint8))
    ds = CityScapes(str(tmp_path / "gtFine") + "/", str(tmp_path / "images"))
    assert len(ds) == 3
    for k in range(3):
        img, lab = ds[k]
        rec = ds.image_dataset[k]
        assert rec.labels[0].endswith("labelTrainIds.png") and rec.labels[1].endswith("color.png")
        assert img.dtype == torch.uint8 and tuple(img.shape) == (8, 16, 3)
        assert lab.dtype == torch.uint8 and tuple(lab.shape) == (8, 16)
    # transforms are applied as the reference applies them (callables on the samples)
    ds2 = CityScapes(str(tmp_path / "gtFine"), str(tmp_path / "images"), transform=lambda t: t.float(),
                     target_transform=lambda t: t.long())
    img, lab = ds2[0]
    assert img.dtype == torch.float32 and lab.dtype == torch.int64


def test_gta5_discovery_and_pairing(tmp_path):
    from rtsds_amd.datasets import GTA5
    rng = np.random.default_rng(1)
    for i in (1, 2, 3):
        _png(tmp_path / "images" / f"{i:05d}.png", rng.integers(0, 256, (6, 10, 3), dtype=np.uint8))
        _png(tmp_path / "labels" / f"{i:05d}.png", rng.integers(0, 19, (6, 10), dtype=np.uint8))
    ds = GTA5(str(tmp_path / "images"), str(tmp_path / "labels"), None, None)
    assert len(ds) == 3
    img, lab = ds[1]
    assert tuple(img.shape) == (6, 10, 3) and tuple(lab.shape) == (6, 10)
    assert ds.images_dataset[1].label[0].endswith("00002.png")


def test_oracle_transform_restatements():
    """The oracle's torchvision restatements: Gaussian kernel normalised and symmetric; the
    integer resize path rounds half-to-even; decode maps each train-id colour to its id."""
    from oracle import transforms as OT
    k = OT._gauss1d(9, 1.7)
    assert abs(float(k.sum()) - 1.0) < 1e-6 and torch.allclose(k, k.flip(0))
    x = torch.tensor([[[0, 1], [1, 0]]], dtype=torch.long)
    y = OT.resize(x, (1, 1))  # mean 0.5 -> rounds to 0 (half to even)
    assert int(y) == 0
    ids = torch.arange(19).view(1, 19)
    rgb = torch.tensor(OT.TRAIN_ID_COLORS).t()[:, ids[0]].view(3, 1, 19)
    assert torch.equal(OT.decode_gta5(rgb), ids)


def test_device_loader_new_permutation_per_iterator():
    """adversarial_train takes next(iter(loader)) every iteration (train.py:186-187);
    with a DistributedSampler each new iterator must draw a new permutation, as the
    reference's RandomSampler does, instead of replaying epoch 0's first batch."""
    from torch.utils.data import DataLoader
    from torch.utils.data.distributed import DistributedSampler
    from rtsds_amd.transforms import DeviceLoader, collate_raw
    ds = [(torch.tensor([i]), torch.tensor([i])) for i in range(64)]
    firsts = {0: [], 1: []}
    for rank in (0, 1):
        sampler = DistributedSampler(ds, num_replicas=2, rank=rank, shuffle=True, seed=3)
        dl = DeviceLoader(DataLoader(ds, batch_size=4, sampler=sampler, collate_fn=collate_raw), lambda t: t, lambda t: t, device="cpu")
        for _ in range(4):
            x, _ = next(iter(dl))
            firsts[rank].append(tuple(int(t) for t in x))
    for rank in (0, 1):
        assert len(set(firsts[rank])) == 4, firsts[rank]
    # the two ranks' shards stay disjoint for each epoch
    for a, b in zip(firsts[0], firsts[1]):
        assert not set(a) & set(b)
