"""Checkpoint interchange that needs no kernels (CPU): the DeepLabV2 pretrained loader's
prefix stripping (reference models/deeplabv2/deeplabv2.py:176-190) and the torch.optim
state_dict format of the rtsds optimizers before their arenas exist."""
import torch

from oracle import models as om
from oracle.weights import apply_recipe


def test_get_deeplab_v2_pretrained_prefix_stripping(tmp_path):
    """A checkpoint whose keys carry one extra leading component ("Scale.conv1.weight", the
    published DeepLab-ResNet ImageNet file's layout) is loaded with weights_only=True, the
    first component stripped and loaded non-strictly: every model key present in the file
    gets its tensor; keys absent from the file (the ASPP head here) keep their init;
    unexpected keys are ignored, as the reference's strict=False load."""
    from rtsds_amd.models.deeplabv2.deeplabv2 import get_deeplab_v2
    src = apply_recipe(om.ResNetMulti(), seed=7)
    saved = {"Scale." + k: v for k, v in src.state_dict().items() if not k.startswith("layer6.")}
    saved["Scale.fc.weight"] = torch.zeros(3)  # no such module: ignored
    path = tmp_path / "DeepLab_resnet_pretrained_imagenet.pth"
    torch.save(saved, path)
    torch.manual_seed(0)
    m = get_deeplab_v2(19, pretrain=True, pretrain_model_path=str(path))
    torch.manual_seed(0)
    fresh = get_deeplab_v2(19, pretrain=False)
    got = m.state_dict()
    for k, v in src.state_dict().items():
        if k.startswith("layer6."):
            assert torch.equal(got[k], fresh.state_dict()[k]), k
        else:
            assert torch.equal(got[k], v), k


def test_state_dict_roundtrip_cpu_models():
    """rtsds modules load a reference-layout state_dict and export it back unchanged (the
    NHWC weight storage is a stride choice: values and shapes are the reference's)."""
    from rtsds_amd.models.bisenet.build_bisenet import BiSeNet
    ref = apply_recipe(om.BiSeNet(19, "resnet18"), seed=11)
    net = BiSeNet(19, "resnet18")
    net.load_state_dict(ref.state_dict())
    back = om.BiSeNet(19, "resnet18")
    back.load_state_dict(net.state_dict())
    for (k, a), (k2, b) in zip(ref.state_dict().items(), back.state_dict().items()):
        assert k == k2 and torch.equal(a, b), k
