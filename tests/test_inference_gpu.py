"""Sliding-window inference on device (reference trainer.py:370-395 -> MONAI sliding_window_inference,
constant blending) against the CPU restatement of MONAI's algorithm in oracle/ with the SAME predictor
(the engine model): windows, accumulation order and normalisation must give bit-identical outputs.
Cases: volume larger than the roi with a clamped last window, exactly one roi, smaller than the roi
(zero padding), batch of 2, overlap 0.5 (the config) and 0.25 (MONAI's default)."""
import pytest
import torch

import mmseg_amd  # noqa: F401
from mmseg_amd.inference import sliding_window_inference
from mmseg_amd.models.build import build_model
from oracle import mmseg_oracle as O

pytestmark = pytest.mark.gpu


def _model(dev):
    cfg = {"data": {"modalities": ["CT", "PET"]},
           "model": {"name": "unet", "in_channels": 2, "out_channels": 3,
                     "backbone": {"features": [8, 16, 32, 64, 128]}, "head": {"dropout": 0.0}},
           "hardware": {"device": "cuda", "engine_dtype": "float32"}}
    torch.manual_seed(0)
    m = build_model(cfg).to(dev)
    m.eval()
    return m


@pytest.mark.parametrize("shape,roi,overlap,swb", [
    ((1, 2, 48, 40, 56), (32, 32, 32), 0.5, 4),     # 3 x 3 x 3 windows, clamped last ones
    ((2, 2, 32, 32, 32), (32, 32, 32), 0.5, 4),     # exactly one roi per image, batch of 2
    ((1, 2, 16, 48, 32), (32, 32, 32), 0.5, 3),     # smaller than the roi along z: zero padding
    ((1, 2, 40, 40, 40), (32, 32, 32), 0.25, 2),    # MONAI's default overlap
])
def test_sliding_window_matches_monai_restatement(dev, shape, roi, overlap, swb):
    m = _model(dev)
    g = torch.Generator().manual_seed(3)
    x = torch.randn(*shape, generator=g).to(dev)
    with torch.no_grad():
        got = sliding_window_inference(x, roi, swb, m, overlap)
        ref = O.sliding_window_inference(x, roi, swb, m, overlap)
    assert got.shape == (shape[0], 3) + shape[2:]
    assert torch.equal(got.cpu(), ref)


def test_trainer_sliding_window_uses_config(dev):
    from mmseg_amd.trainer.trainer import Trainer
    m = _model(dev)
    cfg = dict(m.config)
    cfg["experiment"] = {"name": "swi", "output_dir": "/tmp/mmseg_test_swi", "seed": 0}
    cfg["inference"] = {"sliding_window": {"roi_size": [32, 32, 32], "overlap": 0.5, "mode": "gaussian"},
                        "batch_size": 4}
    cfg["training"] = {"epochs": 1, "optimizer": {"name": "adamw", "lr": 1e-4}, "scheduler": {"name": "none"},
                       "loss": {"name": "dice_ce"}}
    tr = Trainer(cfg, m)
    x = torch.randn(1, 2, 48, 32, 32, generator=torch.Generator().manual_seed(4)).to(dev)
    with torch.no_grad():
        got = tr._sliding_window_inference(x)
        ref = O.sliding_window_inference(x, (32, 32, 32), 4, m, 0.5)
    assert torch.equal(got.cpu(), ref)
