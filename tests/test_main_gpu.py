"""End-to-end CLI (rtsds_amd.main) on synthetic loaders: one DA epoch and one seg epoch at a
small size, BiSeNet and DeepLab generators.  GPU only."""
import pytest
import torch
import yaml

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)

from rtsds_amd import main as rmain  # noqa: E402


def _cfg(tmp_path, gen="bisenet", precision="bf16"):
    cfg = yaml.safe_load(open(rmain.__file__.replace("main.py", "config.yaml")))
    cfg["precision"] = precision
    cfg["data"]["cityscapes"].update(image_size="64, 128", batch_size=2)
    cfg["data"]["gta5_modified"].update(image_size="64, 128", batch_size=2)
    cfg["data"]["synthetic_batches"] = 2
    cfg["training"]["domain_adaptation"].update(iterations=2, epochs=1)
    cfg["training"]["segmentation"].update(epochs=1)
    cfg["model"]["adversarial_model"]["generator"]["name"] = gen
    p = tmp_path / "cfg.yaml"
    p.write_text(yaml.safe_dump(cfg))
    return str(p)


@pytest.mark.parametrize("gen", ["bisenet", "deeplab"])
def test_main_domain_adaptation(tmp_path, monkeypatch, gen):
    monkeypatch.chdir(tmp_path)
    rmain.main(["--config", _cfg(tmp_path, gen), "--domain_adaptation"])


def test_main_segmentation(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    rmain.main(["--config", _cfg(tmp_path, precision="fp32"), "--model", "bisenet"])
