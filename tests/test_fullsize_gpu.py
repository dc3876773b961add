"""Full-size training-step parity: the engine's step at the BASELINE sizes (96^3, B=2) against the reference's
own training step captured by tests/golden/make_golden.py (full_grad_case: reference train-mode forward + loss +
backward, trainer.py:250-254).

Cases: c2 UNet3D CT+PET 6 classes DiceCE; c3 DualEncoder "cross_attention" (= mean fusion, the bench
workload) DiceCE; c5 DualEncoder CT+PET+MRI Tversky.  Each runs in fp32 (the parity path) and in bf16 (the
path bench.py times: brick5 / brick3 / brick2-BN64 with 32-bit staging, wgrad_dma, the fused InstanceNorm
partials, the fused head + loss), through Trainer._fused_loss exactly as Trainer.train_step does.

Compared per parameter tensor, on the fixture's seeded gradient samples (k = 4096 positions, all of them for
smaller tensors): normwise L2 error ||g - g_ref|| / ||g_ref||, and the full-tensor L2 norm against the
reference's.  Conv biases in front of an InstanceNorm have a mathematically zero gradient (pure rounding
noise) and are only bounded in size.

Tolerances:
  * fp32: loss 1e-5 relative; sampled logits 1e-3 normwise (north_star); every gradient 1e-3 normwise (the
    transposed-conv bias, nearly dead, 1e-2); argmax histogram within 1e-4 of the voxels.
  * bf16: activations are stored in bf16 (8 mantissa bits, relative rounding 2^-9 = 2e-3 per store, ~20
    stores deep); loss 2e-3 relative; logits 3e-2 normwise; every gradient 8e-2 normwise and the median over
    tensors 3e-2; gradient norms 5e-2.
"""
import numpy as np
import pytest
import torch

import mmseg_amd  # noqa: F401
from mmseg_amd.models.build import build_model
from mmseg_amd.trainer.trainer import Trainer
from tests.helpers import golden, rel

pytestmark = pytest.mark.gpu

CASES = {
    "fullgrad_unet_c2": ("unet", ["CT", "PET"], "dice_ce"),
    "fullgrad_dual_c3": ("dual_encoder", ["CT", "PET"], "dice_ce"),
    "fullgrad_dual_m3_c5": ("dual_encoder", ["CT", "PET", "MRI"], "tversky"),
}

TOL = {
    "float32": dict(loss=1e-5, logits=1e-3, grad=1e-3, grad_near=1e-2, median=1e-3, norm=1e-3),
    "bfloat16": dict(loss=2e-3, logits=3e-2, grad=8e-2, grad_near=8e-2, median=3e-2, norm=5e-2),
}


def _config(model, mods, loss, dtype):
    return {
        "experiment": {"name": "fullgrad", "output_dir": "/tmp/mmseg_fullgrad", "seed": 0},
        "data": {"modalities": list(mods)},
        "model": {"name": model, "in_channels": len(mods), "out_channels": 6,
                  "backbone": {"features": [32, 64, 128, 256, 512], "norm": "instance"},
                  "fusion": {"type": "cross_attention"}, "head": {"dropout": 0.0}},
        "training": {"epochs": 1, "batch_size": 2, "accumulation_steps": 1,
                     "optimizer": {"name": "adamw", "lr": 1e-4, "weight_decay": 1e-5, "betas": [0.9, 0.999]},
                     "scheduler": {"name": "none"},
                     "loss": {"name": loss, "dice_weight": 0.5, "ce_weight": 0.5, "class_weights": None,
                              "tversky_alpha": 0.5, "tversky_beta": 0.5},
                     "checkpoint": {"save_last": False, "save_best": False}},
        "hardware": {"device": "cuda", "mixed_precision": dtype == "bfloat16", "engine_dtype": dtype},
    }


def full_inputs(S, B, M, C, seed):
    """make_golden.full_inputs: the same seeded data-only inputs."""
    rng = np.random.Generator(np.random.PCG64(seed + 100))
    x = torch.from_numpy(rng.standard_normal((B, M, S, S, S), dtype=np.float32))
    y = torch.from_numpy(rng.integers(0, C, size=(B, S, S, S)).astype(np.int64))
    idx = rng.integers(0, S ** 3, size=1024)
    return x, y, idx


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
@pytest.mark.parametrize("tag", list(CASES))
def test_fullsize_training_step_matches_reference(dev, tag, dtype):
    g = golden(tag)
    model, mods, loss = CASES[tag]
    S, B, seed, C = int(g["S"]), int(g["B"]), int(g["seed"]), 6
    cfg = _config(model, mods, loss, dtype)
    torch.manual_seed(seed)
    m = build_model(cfg)
    names = [n for n, _ in m.backbone.named_parameters()]
    assert names == list(g["param_names"])
    x, y, idx = full_inputs(S, B, len(mods), C, seed)
    assert np.array_equal(idx, g["sample_idx"])
    x, y = x.to(dev), y.to(dev)
    tr = Trainer(cfg, m)
    m.train()
    lossv = tr._fused_loss(x, y)             # the bench's path: fused head + loss node
    assert lossv is not None, "fused head + loss path not taken"
    lossv.backward()
    with torch.no_grad():
        logits = m(x)
    torch.cuda.synchronize()
    t = TOL[dtype]
    ref_loss = float(g["loss"])
    err_loss = abs(lossv.item() - ref_loss) / abs(ref_loss)
    err_logits = rel(logits.reshape(B, C, -1)[:, :, torch.from_numpy(idx).to(dev)],
                     torch.from_numpy(g["sample_logits"]))
    errs, norm_errs, dead_sizes, typical = {}, {}, {}, []
    bb = dict(m.backbone.named_parameters())
    off = g["gs_off"]
    for i, n in enumerate(names):
        gi = torch.from_numpy(g["gs_idx"][off[i]:off[i + 1]]).to(dev)
        gref = torch.from_numpy(g["gs_val"][off[i]:off[i + 1]])
        geng = bb[n].grad.reshape(-1)[gi].double().cpu()
        if n.endswith(("conv1.bias", "conv2.bias")):
            dead_sizes[n] = float(geng.norm())
            continue
        errs[n] = float((geng - gref).norm() / gref.norm())
        norm_errs[n] = abs(float(bb[n].grad.double().norm()) - float(g["grad_norm"][i])) / float(g["grad_norm"][i])
        typical.append(float(g["grad_norm"][i]) / np.sqrt(bb[n].numel()))
    med = float(np.median(list(errs.values())))
    worst = sorted(((v, n) for n, v in errs.items()), reverse=True)[:5]
    print(f"\n{tag} {dtype}: loss {lossv.item():.7f} vs {ref_loss:.7f} (rel {err_loss:.2e}), logits {err_logits:.2e}, "
          f"grad median {med:.2e}, worst {[(round(v, 5), n) for v, n in worst]}, "
          f"norm worst {max(norm_errs.values()):.2e}")
    assert err_loss < t["loss"], err_loss
    assert err_logits < t["logits"], err_logits
    bad = {n: v for n, v in errs.items() if v > (t["grad_near"] if n.endswith("up.bias") else t["grad"])}
    assert not bad, bad
    assert med < t["median"], med
    bad = {n: v for n, v in norm_errs.items() if v > (t["grad_near"] if n.endswith("up.bias") else t["norm"])}
    assert not bad, bad
    # mathematically-zero gradients stay at the rounding-noise scale of the live ones
    scale = float(np.median(typical)) * np.sqrt(4096)
    assert all(v < 1e-2 * scale for v in dead_sizes.values()), dead_sizes
    if dtype == "float32":
        hist = torch.bincount(logits.argmax(1).reshape(-1), minlength=C).cpu().numpy()
        assert np.abs(hist - g["argmax_hist"]).sum() <= 1e-4 * hist.sum()
