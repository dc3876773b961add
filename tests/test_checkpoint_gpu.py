"""Checkpoint / resume compatibility with the reference and the `main.py --mode train` drop-in (config c1).

  * A checkpoint WRITTEN BY THE REFERENCE (tests/golden/make_golden.py checkpoint_case: reference
    save_checkpoint, build.py:153-180, after 2 Trainer steps) is read with the safe loader and resumed through
    Trainer(resume_from=...) (reference trainer.py:150-164); the next training step must give the reference's
    next-step loss and parameters.
  * `main.main(["--mode", "train", ...])` (reference main.py:310-339, 501-549) on config c1 (UNet3D CT+PET 64^3,
    batch 1, 3 classes, DiceCE) writes last.pth / best.pth in the reference's format: the same top-level keys,
    the same model state-dict keys and shapes as the reference's c1 model, torch AdamW optimizer state; and
    `--resume` from it trains on.
"""
import os

import numpy as np
import pytest
import torch
import yaml

import mmseg_amd  # noqa: F401
from mmseg_amd.models.build import build_model
from mmseg_amd.trainer.trainer import Trainer
from tests.helpers import GOLDEN, golden

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_CKPT = os.path.join(GOLDEN, "ref_ckpt_unet_small.pth")


def _small_cfg(tmp):
    return {
        "experiment": {"name": "ckpt", "output_dir": str(tmp), "seed": 0},
        "data": {"modalities": ["CT", "PET"]},
        "model": {"name": "unet", "in_channels": 2, "out_channels": 3,
                  "backbone": {"features": [8, 16, 32], "norm": "instance"},
                  "fusion": {"type": "cross_attention"}, "head": {"dropout": 0.0}},
        "training": {"epochs": 1, "batch_size": 2, "accumulation_steps": 1,
                     "optimizer": {"name": "adamw", "lr": 1e-3, "weight_decay": 1e-5, "betas": [0.9, 0.999]},
                     "scheduler": {"name": "none"},
                     "loss": {"name": "dice_ce", "dice_weight": 0.5, "ce_weight": 0.5, "class_weights": None},
                     "checkpoint": {"save_last": False, "save_best": False}},
        "hardware": {"device": "cuda", "mixed_precision": False, "engine_dtype": "float32"},
    }


def test_resume_from_reference_checkpoint(dev, tmp_path):
    g = golden("ref_ckpt_unet_small")
    ck = torch.load(REF_CKPT, map_location="cpu", weights_only=True)
    assert set(ck) == {"epoch", "model_state_dict", "optimizer_state_dict", "best_metric", "history"}
    cfg = _small_cfg(tmp_path)
    torch.manual_seed(123)                      # a different init: everything must come from the file
    m = build_model(cfg)
    tr = Trainer(cfg, m, resume_from=REF_CKPT)
    assert tr.current_epoch == int(g["resume_epoch"]) and tr.best_metric == 0.25
    gen = torch.Generator().manual_seed(31)
    xs = torch.randn(3, 2, 2, 32, 32, 32, generator=gen)
    ys = torch.randint(0, 3, (3, 2, 32, 32, 32), generator=gen)
    loss = tr.train_step({"image": xs[2], "label": ys[2]}, 0)
    assert abs(loss - float(g["next_loss"])) < 1e-5, (loss, float(g["next_loss"]))
    names = [n for n, _ in m.named_parameters()]
    assert names == list(g["names"])
    after = torch.cat([p.detach().reshape(-1).double().cpu() for p in m.parameters()]).numpy()
    ref = g["after"]
    live = np.concatenate([np.full(p.numel(), not n.endswith(("conv1.bias", "conv2.bias")))
                           for n, p in m.named_parameters()])
    # the resumed moments and step count (2 -> 3) drive the update: live weights within fp32 rounding of the
    # reference's; the biases in front of an InstanceNorm have a gradient of pure rounding noise, so their
    # AdamW update is ~lr * noise-sign: bounded by a few lr
    assert np.linalg.norm(after[live] - ref[live]) / np.linalg.norm(ref[live]) < 1e-6
    assert np.abs(after[live] - ref[live]).max() < 1e-5
    assert np.abs(after[~live] - ref[~live]).max() < 3e-3


def test_engine_checkpoint_matches_reference_format(dev, tmp_path):
    """An engine-written checkpoint has the reference checkpoint's structure (the reference's own .pth is the
    template), so the reference's load_checkpoint / _resume can read it."""
    ref = torch.load(REF_CKPT, map_location="cpu", weights_only=True)
    cfg = _small_cfg(tmp_path)
    cfg["training"]["checkpoint"] = {"save_last": True, "save_best": True}
    torch.manual_seed(0)
    m = build_model(cfg)
    tr = Trainer(cfg, m)
    gen = torch.Generator().manual_seed(31)
    tr.train_step({"image": torch.randn(2, 2, 32, 32, 32, generator=gen),
                   "label": torch.randint(0, 3, (2, 32, 32, 32), generator=gen)}, 0)
    tr.history = {"train_loss": [1.0], "val_loss": [1.1], "val_dice": [0.25]}
    tr._save_checkpoints({"dice": 0.5})
    for name in ("last.pth", "best.pth"):
        ck = torch.load(tmp_path / "ckpt" / name, map_location="cpu", weights_only=True)
        assert set(ck) == set(ref)
        assert list(ck["model_state_dict"]) == list(ref["model_state_dict"])
        for k, v in ref["model_state_dict"].items():
            assert ck["model_state_dict"][k].shape == v.shape and ck["model_state_dict"][k].dtype == v.dtype
        so, ro = ck["optimizer_state_dict"], ref["optimizer_state_dict"]
        assert set(so) == set(ro) and set(so["state"]) == set(ro["state"])
        for i, st in ro["state"].items():
            assert set(so["state"][i]) == set(st)
            for k, v in st.items():
                assert so["state"][i][k].shape == v.shape and so["state"][i][k].dtype == v.dtype, (i, k)
        assert [sorted(pg) for pg in so["param_groups"]] == [sorted(pg) for pg in ro["param_groups"]]
    # and it round-trips into a fresh engine model
    torch.manual_seed(5)
    m2 = build_model(cfg)
    tr2 = Trainer(cfg, m2, resume_from=str(tmp_path / "ckpt" / "last.pth"))
    for a, b in zip(m.parameters(), m2.parameters()):
        assert torch.equal(a.detach().cpu(), b.detach().cpu())
    assert int(tr2.optimizer.state[next(m2.parameters())]["step"]) == 1


@pytest.mark.parametrize("device_data", [False, True])
def test_main_train_c1(dev, tmp_path, device_data):
    """python main.py --mode train --config configs/c1_unet_64_cpu_plumbing.yaml (BASELINE configs[0]) through
    main.main(argv), 1 epoch over 8 phantoms (host numpy phantoms, or generated + normalised on the device);
    then --resume from the written last.pth for a second epoch."""
    import main as entry
    with open(os.path.join(ROOT, "configs", "c1_unet_64_cpu_plumbing.yaml")) as f:
        cfg = yaml.safe_load(f)
    cfg["experiment"]["log_dir"] = str(tmp_path / "logs")
    cfg["data"]["synthetic"]["device"] = device_data
    cpath = tmp_path / "c1.yaml"
    with open(cpath, "w") as f:
        yaml.safe_dump(cfg, f)
    out = tmp_path / "out"
    entry.main(["--mode", "train", "--config", str(cpath), "--epochs", "1", "--output-dir", str(out)])
    g = golden("ref_ckpt_unet_small")
    d = out / cfg["experiment"]["name"]
    for name in ("last.pth", "best.pth"):
        ck = torch.load(d / name, map_location="cpu", weights_only=True)
        assert set(ck) == {"epoch", "model_state_dict", "optimizer_state_dict", "best_metric", "history"}
        assert list(ck["model_state_dict"]) == list(g["c1_unet_keys"])
        shapes = [",".join(map(str, v.shape)) for v in ck["model_state_dict"].values()]
        assert shapes == list(g["c1_unet_shapes"])
        assert len(ck["history"]["train_loss"]) == 1 and np.isfinite(ck["history"]["train_loss"][0])
        assert 0.0 <= ck["history"]["val_dice"][0] <= 1.0
    # reference quirk kept: _resume sets current_epoch = ckpt["epoch"], so the saved epoch runs again
    entry.main(["--mode", "train", "--config", str(cpath), "--epochs", "2", "--output-dir", str(out),
                "--resume", str(d / "last.pth")])
    ck = torch.load(d / "last.pth", map_location="cpu", weights_only=True)
    assert ck["epoch"] == 1
