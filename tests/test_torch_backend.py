"""hardware.kernels: torch -- the A/B backend SURVEY §8b keeps selectable: the same parameter containers and
losses through plain PyTorch ops (the reference's own module forward, unet.py:53-60 / 74-79 / 104-113 /
165-200, dual_encoder.py:112-199 / 243-254, losses.py:47-228).

CPU tests pin its arithmetic to the reference's golden fixtures (tests/golden/make_golden.py) by calling the
torch-op forwards directly: the product entry points (model(x), criterion(...)) refuse CPU tensors, like the HIP
backend.  GPU tests compare the two backends on the device through the drop-in API."""
import copy

import numpy as np
import pytest
import torch

import mmseg_amd  # noqa: F401
from mmseg_amd.models.build import build_model
from mmseg_amd.trainer.losses import get_loss
from tests.helpers import golden, rel
from tests.test_model_gpu import TINY, _inputs, make_config

torch.set_num_threads(min(8, torch.get_num_threads()))


def _build_cpu(tag, kernels="torch"):
    model, mods, C, fusion, loss = TINY[tag]
    g = golden(tag)
    cfg = make_config(model, mods, C, list(g["features"]), fusion=fusion, loss=loss)
    cfg["hardware"]["device"] = "cpu"
    cfg["hardware"]["kernels"] = kernels
    torch.manual_seed(int(g["seed"]))
    m = build_model(cfg)
    return cfg, m, g, len(mods), C


@pytest.mark.parametrize("tag", list(TINY))
def test_torch_backend_matches_reference_goldens(tag):
    cfg, m, g, M, C = _build_cpu(tag)
    bb = m.backbone
    xs, ys = _inputs(g, M, C)
    bb.train()
    out = bb.torch_forward(xs[0])
    crit = get_loss(cfg)
    assert crit.kernels == "torch"
    loss = crit.torch_forward(out, ys[0])
    loss.backward()
    flat = out.detach().reshape(-1)
    assert rel(flat[torch.from_numpy(g["sample_idx"])], torch.from_numpy(g["sample_logits"])) < 1e-5
    assert abs(loss.item() - float(g["loss"])) < 1e-6
    names = list(g["init_names"])
    params = dict(bb.named_parameters())
    gn = np.array([params[n].grad.double().norm().item() for n in names])
    live = gn > 1e-6 * gn.max()
    assert np.allclose(gn[live], g["grad_norm"][live], rtol=1e-4)


@pytest.mark.parametrize("C", [3, 6])
def test_torch_losses_match_reference_goldens(C):
    from mmseg_amd.trainer import losses as L
    g = golden("losses")
    logits = torch.from_numpy(g[f"logits_C{C}"])
    labels = torch.from_numpy(g[f"labels_C{C}"]).long()
    cw = torch.from_numpy(g[f"cw_C{C}"])
    cases = {"dicece": L.DiceCELoss(), "dicece_w": L.DiceCELoss(0.3, 0.7, class_weights=cw), "dice": L.DiceLoss(),
             "dice_nobg": L.DiceLoss(include_background=False), "ce": L.CrossEntropyLoss(),
             "tversky": L.TverskyLoss(), "tversky_37": L.TverskyLoss(alpha=0.3, beta=0.7), "focal": L.FocalLoss(),
             "focal_w": L.FocalLoss(alpha=cw)}
    for name, crit in cases.items():
        x = logits.clone().requires_grad_(True)
        loss = crit.torch_forward(x, labels)
        loss.backward()
        assert abs(loss.item() - float(g[f"{name}_C{C}"])) < 1e-6, name
        assert rel(x.grad, torch.from_numpy(g[f"{name}_C{C}_grad"])) < 1e-5, name


def test_torch_backend_refuses_cpu_and_unknown_names():
    cfg, m, g, M, C = _build_cpu("unet_tiny")
    xs, ys = _inputs(g, M, C)
    with pytest.raises(RuntimeError, match="no CPU path"):
        m(xs[0])
    with pytest.raises(RuntimeError, match="no CPU path"):
        get_loss(cfg)(torch.zeros(1, C, 2, 2, 2), torch.zeros(1, 2, 2, 2, dtype=torch.long))
    bad = copy.deepcopy(cfg)
    bad["hardware"]["kernels"] = "triton"
    with pytest.raises(ValueError, match="hardware.kernels"):
        build_model(bad)


def test_torch_backend_not_for_swin():
    cfg = make_config("swin_unetr", ["CT", "PET"], 3, [32, 64])
    cfg["model"]["backbone"] = {"img_size": [32, 32, 32], "feature_size": 12}
    cfg["hardware"]["device"] = "cpu"
    cfg["hardware"]["kernels"] = "torch"
    with pytest.raises(ValueError, match="kernels: torch"):
        build_model(cfg)


# ------------------------------------------------------------------ GPU: the two backends side by side
@pytest.mark.gpu
@pytest.mark.parametrize("tag", ["unet_tiny", "dual_tiny_cross_attention", "dual_tiny_attention",
                                 "dual_tiny_m3_tversky"])
def test_torch_and_hip_backends_agree_on_gpu(dev, tag):
    """fp32: the HIP program and PyTorch-ROCm (MIOpen) on the same weights and batch: logits, loss and the
    3-step Trainer trajectory (torch.optim.AdamW vs FlatAdamW)."""
    from mmseg_amd.trainer.trainer import Trainer
    res = {}
    for kernels in ("hip", "torch"):
        model, mods, C, fusion, loss = TINY[tag]
        g = golden(tag)
        cfg = make_config(model, mods, C, list(g["features"]), fusion=fusion, loss=loss)
        cfg["hardware"]["kernels"] = kernels
        torch.manual_seed(int(g["seed"]))
        m = build_model(cfg)
        xs, ys = _inputs(g, len(mods), C)
        m.eval()
        with torch.no_grad():
            logits = m(xs[0].to(dev)).cpu()
        tr = Trainer(cfg, m)
        traj = [tr.train_step({"image": xs[1 + i], "label": ys[1 + i]}, i) for i in range(int(g["steps"]))]
        res[kernels] = (logits, traj)
    assert rel(res["hip"][0], res["torch"][0]) < 1e-4
    assert np.allclose(res["hip"][1], res["torch"][1], rtol=0, atol=1e-4), (res["hip"][1], res["torch"][1])
    assert np.allclose(res["torch"][1], golden(tag)["traj_losses"], rtol=0, atol=1e-4)


@pytest.mark.gpu
def test_torch_backend_amp_step_runs(dev):
    """The reference's GPU mode (fp16 autocast + GradScaler) and bf16 autocast on the torch backend: finite
    decreasing-or-equal-order losses on a tiny DualEncoder."""
    from mmseg_amd.trainer.trainer import Trainer
    for edt in ("float32", "bfloat16"):
        model, mods, C, fusion, loss = TINY["dual_tiny_cross_attention"]
        g = golden("dual_tiny_cross_attention")
        cfg = make_config(model, mods, C, list(g["features"]), fusion=fusion, loss=loss, dtype=edt)
        cfg["hardware"]["kernels"] = "torch"
        cfg["hardware"]["mixed_precision"] = True
        torch.manual_seed(int(g["seed"]))
        m = build_model(cfg)
        tr = Trainer(cfg, m)
        assert (tr.scaler is not None) == (edt == "float32")
        xs, ys = _inputs(g, len(mods), C)
        losses = [tr.train_step({"image": xs[1], "label": ys[1]}, i) for i in range(3)]
        assert all(np.isfinite(losses))
        assert abs(losses[0] - float(g["loss"])) < 5e-2


def test_fp8_config_checks():
    """hardware.fp8 (config c5's mixed bf16/fp8) needs the HIP backend with bf16 storage."""
    cfg = make_config("dual_encoder", ["CT", "PET", "MRI"], 4, [32, 64], loss="tversky", dtype="float32")
    cfg["hardware"]["fp8"] = True
    cfg["hardware"]["device"] = "cpu"
    with pytest.raises(ValueError, match="fp8"):
        build_model(cfg)
    cfg["hardware"]["engine_dtype"] = "bfloat16"
    cfg["hardware"]["kernels"] = "torch"
    with pytest.raises(ValueError, match="fp8"):
        build_model(cfg)
