"""Device-side data path (csrc/data.hip) against the reference's own transforms and the CPU
oracle: ModalitySpecificNormalize (transforms.py:362-404) and Resize (transforms.py:215-250) on the golden raw
CT/PET/MRI sample the reference processed (tests/golden/transforms.npz): CT / PET bit-identical, MRI z-score and
the trilinear resize within 1 float32 ulp-level (2e-7 relative), labels bit-identical; the device phantom
generator against its restatement in oracle/data_oracle.py (labels bit-identical, intensities 1e-6)."""
import numpy as np
import pytest
import torch

import mmseg_amd  # noqa: F401
from mmseg_amd.data.device import (DeviceLoader, DeviceModalityNormalize, DevicePhantomDataset, DeviceResize,
                                   device_phantom, phantom_params)
from mmseg_amd.data.dataloader import get_dataloader
from oracle import data_oracle as DO
from tests.helpers import golden

pytestmark = pytest.mark.gpu
PRE = {"ct": {"window_center": -100, "window_width": 700}, "pet": {"normalize": True}, "mri": {"normalize": True}}


def test_normalize_matches_reference(dev):
    g = golden("transforms")
    img = torch.from_numpy(g["image_in"]).to(dev).contiguous()
    DeviceModalityNormalize({"data": {"modalities": ["CT", "PET", "MRI"], "preprocessing": PRE}})(img)
    got, ref = img.cpu().numpy(), g["normalized"]
    assert np.array_equal(got[0], ref[0])          # CT window: float32 arithmetic, bit-identical
    assert np.array_equal(got[1], ref[1])          # PET / max
    assert np.abs(got[2] - ref[2]).max() <= 2e-7 * np.abs(ref[2]).max()


@pytest.mark.parametrize("name", ["up", "down"])
def test_resize_matches_reference(dev, name):
    g = golden("transforms")
    size = tuple(int(v) for v in g[f"size_{name}"])
    sample = {"image": torch.from_numpy(g["normalized"]).to(dev), "label": torch.from_numpy(g["label_in"]).to(dev)}
    out = DeviceResize(size)(sample)
    ref = g[f"resized_{name}"]
    assert out["image"].shape == ref.shape
    assert np.abs(out["image"].cpu().numpy() - ref).max() <= 2e-7 * np.abs(ref).max()
    assert np.array_equal(out["label"].cpu().numpy(), g[f"label_{name}"])


@pytest.mark.parametrize("mods,C,S", [(["CT", "PET"], 6, 24), (["CT", "PET", "MRI"], 3, 17)])
def test_phantom_matches_oracle(dev, mods, C, S):
    seed = 4321
    img, lab = device_phantom(seed, S, C, mods, dev)
    geo, means, sds, absn, keys = phantom_params(seed, S, C, mods)
    ref_lab = DO.phantom_labels(S, geo[:, :3], geo[:, 3:])
    assert np.array_equal(lab.cpu().numpy(), ref_lab)
    assert len(np.unique(ref_lab)) > 1
    for m in range(len(mods)):
        ref = DO.phantom_intensity(ref_lab, means[m], float(sds[m]), int(keys[m]), bool(absn[m]))
        got = img[m].cpu().numpy()
        assert np.abs(got - ref).max() <= 1e-6 * max(1.0, np.abs(ref).max())


def test_device_loader_batches(dev):
    ds = DevicePhantomDataset(5, 32, 4, ["CT", "PET"], dev, seed=7)
    ld = DeviceLoader(ds, 2, shuffle=True, drop_last=True)
    assert len(ld) == 2
    batches = list(ld)
    b = batches[0]
    assert b["image"].shape == (2, 2, 32, 32, 32) and b["image"].device.type == "cuda"
    assert b["label"].shape == (2, 32, 32, 32) and b["label"].dtype == torch.int64
    assert b["CT"].shape == (2, 1, 32, 32, 32) and len(b["patient_id"]) == 2
    ct, pet = b["image"][:, 0], b["image"][:, 1]
    assert ct.min() >= 0 and ct.max() <= 1                     # CT window -> [0, 1]
    assert torch.allclose(pet.amax(dim=(1, 2, 3)), torch.ones(2, device=dev))   # PET / max
    # the same sample twice is the same tensor (counter-based noise)
    a0 = ds[3]["image"]
    assert torch.equal(a0, ds[3]["image"])


def test_get_dataloader_device_flag(dev):
    cfg = {"data": {"modalities": ["CT", "PET"], "synthetic": {"n_train": 4, "n_val": 2, "size": 32, "seed": 11,
                                                             "device": True}},
           "model": {"out_channels": 3}, "training": {"batch_size": 2}, "hardware": {}}
    ld = get_dataloader(cfg, "train")
    assert isinstance(ld, DeviceLoader) and len(ld) == 2
    b = next(iter(ld))
    assert b["image"].is_cuda and b["label"].max() < 3


def test_trainer_epoch_on_device_loader(dev):
    """Trainer._train_epoch / _validate over the device loader (UNet3D, tiny features, 32^3)."""
    from bench import make_config
    from mmseg_amd.models.build import build_model
    from mmseg_amd.trainer.trainer import Trainer
    cfg = make_config("unet", 2, "bf16", out_channels=3)
    cfg["model"]["backbone"]["features"] = [8, 16, 32, 64, 128]
    cfg["data"]["synthetic"] = {"n_train": 4, "n_val": 2, "size": 32, "seed": 5, "device": True}
    torch.manual_seed(0)
    model = build_model(cfg)
    tr = Trainer(cfg, model, train_loader=get_dataloader(cfg, "train"), val_loader=get_dataloader(cfg, "val"))
    loss = tr._train_epoch()
    vloss, met = tr._validate()
    assert np.isfinite(loss) and np.isfinite(vloss) and 0.0 <= met["dice"] <= 1.0
