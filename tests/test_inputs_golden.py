"""The reference's input-pipeline code that needs no torchvision kernel, pinned by fixtures
captured from the imported reference (tests/golden/make_golden.py --only inputs ->
tests/golden/inputs.{npz,json}):

* GTA5.__decode_label__ (datasets/gta5.py:111-119; colour map :10-46): every colour of the map
  (ignore classes -> 0, car / license plate and pole / polegroup sharing a colour), near-miss and
  random colours -> 0;
* IntRangeTransformer(0, 19) (utils.py:67-75) on int64 and float labels;
* CityScapes.__merge_ids__ (datasets/cityscapes.py:31-50) and GTA5.__make_dataset__
  (datasets/gta5.py:85-100) on the same file lists.

CPU: the oracle restatement and the product's host code vs the fixtures.  The device kernels
(rtsds_gta5_decode, the label resize's clamp) are checked against the same fixtures in
tests/test_transforms_gpu.py.  torchvision's antialiased Resize / Normalize stay "parity
unpinned" (torchvision is absent; tests/test_transforms_gpu.py checks them against
oracle/transforms.py)."""
import types

import torch

from oracle import transforms as OT
from rtsds_amd.datasets.cityscapes import CityScapes
from rtsds_amd.datasets.gta5 import GTA5, TRAIN_ID_COLORS
from rtsds_amd.utils import IntRangeTransformer


def test_gta5_decode_oracle_matches_reference(golden):
    arrays, meta = golden("inputs")
    rgb = torch.from_numpy(arrays["gta5_rgb"])
    want = torch.from_numpy(arrays["gta5_ids"]).long()
    assert meta["gta5_ids_shape"] == [1, *want.shape]
    got = OT.decode_gta5(rgb.permute(2, 0, 1).long())
    assert torch.equal(got, want)
    # the product's colour table is the reference's first colour per train id
    pal = {tuple(c) for c in meta["gta5_palette"]}
    assert all(tuple(c) in pal for c in TRAIN_ID_COLORS)
    for i, col in enumerate(TRAIN_ID_COLORS):
        hit = (rgb == torch.tensor(col, dtype=torch.uint8)).all(-1)
        assert hit.any() and bool((want[hit] == i).all()), i


def test_int_range_matches_reference(golden):
    arrays, _ = golden("inputs")
    clamp = IntRangeTransformer(min_val=0, max_val=19)
    for kind in ("long", "float"):
        x = torch.from_numpy(arrays["int_range_in_" + kind])
        x = x.long() if kind == "long" else x
        want = torch.from_numpy(arrays["int_range_out_" + kind]).long()
        got = clamp(x)
        assert got.dtype == torch.int64 and torch.equal(got, want), kind
        assert torch.equal(OT.int_range(x, 0, 19), want), kind


def test_cityscapes_merge_matches_reference(golden):
    _, meta = golden("inputs")
    m = meta["cityscapes"]
    cs = types.SimpleNamespace(images_filename=list(m["images"]), annotations_filename=list(m["annotations"]))
    got = [[r.path, list(r.labels)] for r in CityScapes.__merge_ids__(cs)]
    assert got == m["merged"]


def test_gta5_make_dataset_matches_reference(golden):
    _, meta = golden("inputs")
    m = meta["gta5_dataset"]
    gt = types.SimpleNamespace(images_filenames=list(m["images"]), labels_filenames=list(m["labels"]))
    got = [[r.image, list(r.label)] for r in GTA5.__make_dataset__(gt)]
    assert got == m["pairs"]
