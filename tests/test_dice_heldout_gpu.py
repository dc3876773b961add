"""north_star: "Dice on a held-out synthetic set matching reference +-1e-4" (BASELINE.json metric "+ Dice vs ref").

The reference's run is in tests/golden/dice_heldout_c1.npz (make_golden.py dice_heldout_case): config c1
(UNet3D CT+PET, 3 classes, 64^3, batch 1, DiceCE, AdamW lr 1e-4), one epoch over K = 16 seeded phantoms
(train seeds 1234..1249, reference trainer.py:222-263), then _validate (trainer.py:265-296, DiceMetric
metrics.py:42-88) on 2 held-out phantoms (seeds 4321, 4322).  The engine runs the same epoch through
Trainer.train_step and validates through Trainer._validate (on-device argmax + counts).

What is compared, and why the Dice bound is what it is:
  * training losses: within 5e-5 at every step (the reference's own fp32-vs-fp64 runs differ by 7.8e-6);
  * held-out validation loss: within 1e-5 (reference fp32 vs fp64: 4.5e-9);
  * held-out Dice (foreground mean): within max(1e-4, 2 |ref_fp32 - ref_fp64|).  A free-running 16-step
    trajectory amplifies rounding (AdamW's first steps move weights by ~lr*sign(g) wherever g is tiny), and
    the model predicts few class-2 voxels (877 of 22132 in the union), so 4 voxels of intersection move the
    Dice by 3.6e-4: the reference against ITSELF in fp64 differs by 3.6e-4.  A +-1e-4 bound on the
    free-running Dice is below the reference's own reproducibility;
  * the Dice itself, given the argmax masks: the engine's model after the same 16 steps is evaluated by the
    oracle (the torch-CPU restatement pinned to the reference, oracle/mmseg_oracle.py) on the same held-out
    volumes; argmax flips between the engine's and the oracle's masks are counted and reported, and the
    engine's on-device Dice counts on its own masks are bit-identical to DiceMetric's on the same masks.
"""
import numpy as np
import pytest
import torch

import mmseg_amd  # noqa: F401
from mmseg_amd.data.synthetic import phantom
from mmseg_amd.models.build import build_model
from mmseg_amd.trainer.metrics import DiceMetric
from mmseg_amd.trainer.trainer import Trainer
from tests.helpers import golden

pytestmark = pytest.mark.gpu


def envelope(case: str, g) -> tuple:
    """The reference's own reproducibility envelope of a free-running held-out Dice (make_golden.py
    dice_heldout_envelope_case): its fp32 run at 1, 2, 4, 6 and 8 intra-op threads (each thread count is another
    summation order of the same algorithm) and its fp64 run.  A correct fp32 implementation with yet another
    summation order -- the HIP engine -- lands somewhere in this spread, so the gate is the envelope widened by half
    its width (at least 1e-4): no legitimate reordering can flip it, while a real error (a wrong gradient, a lost
    update) moves the trajectory far outside it.  Returns (lo, hi, values)."""
    e = golden("dice_heldout_envelope")
    vals = np.concatenate([e[f"{case}_f32_dice"], [float(g["f32_dice"]), float(g["f64_dice"])]])
    w = max(float(vals.max() - vals.min()), 1e-4)
    return float(vals.min()) - 0.5 * w, float(vals.max()) + 0.5 * w, vals


def _cfg():
    return {
        "experiment": {"name": "heldout", "output_dir": "/tmp/mmseg_heldout", "seed": 42},
        "data": {"modalities": ["CT", "PET"]},
        "model": {"name": "unet", "in_channels": 2, "out_channels": 3,
                  "backbone": {"features": [32, 64, 128, 256, 512], "norm": "instance"},
                  "fusion": {"type": "cross_attention"}, "head": {"dropout": 0.0}},
        "training": {"epochs": 1, "batch_size": 1, "accumulation_steps": 1,
                     "optimizer": {"name": "adamw", "lr": 1e-4, "weight_decay": 1e-5, "betas": [0.9, 0.999]},
                     "scheduler": {"name": "none"},
                     "loss": {"name": "dice_ce", "dice_weight": 0.5, "ce_weight": 0.5, "class_weights": None},
                     "checkpoint": {"save_last": False, "save_best": False}},
        "hardware": {"device": "cuda", "mixed_precision": False, "engine_dtype": "float32"},
    }


def _batch(seed, S):
    p = phantom(int(seed), S, 3, ["CT", "PET"])
    return {"image": torch.from_numpy(np.stack([p["CT"], p["PET"]]))[None],
            "label": torch.from_numpy(p["label"])[None]}


def test_heldout_dice_matches_reference(dev):
    from oracle import mmseg_oracle as O
    g = golden("dice_heldout_c1")
    S = int(g["S"])
    cfg = _cfg()
    torch.manual_seed(42)
    m = build_model(cfg)
    train = [_batch(s, S) for s in g["train_seeds"]]
    val = [_batch(s, S) for s in g["val_seeds"]]
    tr = Trainer(cfg, m, val_loader=val)
    m.train()
    losses = np.array([tr.train_step(b, i) for i, b in enumerate(train)])
    vloss, met = tr._validate()
    ref_dice, ref64 = float(g["f32_dice"]), float(g["f64_dice"])
    spread = abs(ref_dice - ref64)
    # teacher-forced metric check: the oracle evaluates the engine's trained weights on the same volumes
    params = {n[len("backbone."):]: p.detach().cpu().float() for n, p in m.named_parameters()}
    dm_eng, dm_orc = DiceMetric(num_classes=3), DiceMetric(num_classes=3)
    flips = 0
    m.eval()
    with torch.no_grad():
        for b in val:
            pe = m(b["image"].to(dev)).argmax(1)
            po = O.unet3d_forward(params, b["image"]).argmax(1)
            flips += int((pe.cpu() != po).sum())
            dm_eng.update(pe, b["label"].to(dev))
            dm_orc.update(po.to(dev), b["label"].to(dev))
    res_eng = dm_eng.compute()
    nvox = len(val) * S ** 3
    print(f"\nheld-out Dice: engine {met['dice']:.6f}, reference fp32 {ref_dice:.6f}, reference fp64 {ref64:.6f} "
          f"(|engine - ref| {abs(met['dice'] - ref_dice):.2e}, reference's own spread {spread:.2e}); per class "
          f"{np.round(met['dice_per_class'], 6).tolist()} vs {np.round(g['f32_dice_per_class'], 6).tolist()}; "
          f"val loss {vloss:.8f} vs {float(g['f32_val_loss']):.8f}; train loss max diff "
          f"{np.abs(losses - g['f32_train_losses']).max():.2e}; argmax flips engine vs oracle on the engine's "
          f"weights: {flips} of {nvox} voxels, oracle Dice {dm_orc.compute()['dice']:.6f}")
    lo, hi, vals = envelope("c1", g)
    print(f"reference envelope (fp32 at 1/2/4/6/8 threads, fp64): {np.round(vals, 6).tolist()}; gate [{lo:.6f}, "
          f"{hi:.6f}], margin {min(met['dice'] - lo, hi - met['dice']):.2e}")
    assert np.abs(losses - g["f32_train_losses"]).max() < 5e-5
    assert abs(vloss - float(g["f32_val_loss"])) < 1e-5
    assert lo <= met["dice"] <= hi
    # _validate's on-device fused argmax + counts == DiceMetric.update on the engine's own masks, bit for bit
    assert met["dice"] == res_eng["dice"] and met["dice_per_class"] == res_eng["dice_per_class"]
    assert flips <= 1e-4 * nvox


# ---------------------------------------------------------------------------------------------------------------
# Held-out Dice on the REFERENCE's trained weights (make_golden.py dice_heldout_trained_case)
# ---------------------------------------------------------------------------------------------------------------
def _trained_cfg(g):
    cfg = _cfg()
    cfg["model"]["backbone"]["features"] = [int(f) for f in g["features"]]
    cfg["training"]["optimizer"]["lr"] = float(g["lr"])
    return cfg


def _trained_batch(g, seed):
    p = phantom(int(seed), int(g["S"]), 3, ["CT", "PET"], class_seed=int(g["class_seed"]))
    return {"image": torch.from_numpy(np.stack([p["CT"], p["PET"]]))[None],
            "label": torch.from_numpy(p["label"])[None]}


def test_heldout_dice_on_reference_weights(dev):
    """The reference trained a UNet3D (CT+PET, 3 classes, 64^3, features 8..128) for K = 160 AdamW steps on
    organ-consistent phantoms (the organs' intensities are the same in every phantom, so it learns which organ
    is which: held-out foreground Dice 0.93) and scored V = 16 held-out phantoms (4.2 M voxels) with its own
    _validate (trainer.py:265-296, DiceMetric metrics.py:42-88).  The engine loads those weights and runs ITS
    _validate (fused on-device argmax + counts): the Dice must match to +-1e-4 (north_star); argmax flips against
    the reference's stored masks are counted and reported."""
    g = golden("dice_heldout_trained")
    cfg = _trained_cfg(g)
    torch.manual_seed(0)
    m = build_model(cfg)
    names = [n for n, _ in m.named_parameters()]
    assert names == list(g["param_names"])
    with torch.no_grad():
        for i, (n, p) in enumerate(m.named_parameters()):
            p.copy_(torch.from_numpy(g[f"w{i}"]).to(dev))
    val = [_trained_batch(g, s) for s in g["val_seeds"]]
    tr = Trainer(cfg, m, val_loader=val)
    vloss, met = tr._validate()
    flips = 0
    m.eval()
    with torch.no_grad():
        for i, b in enumerate(val):
            pe = m(b["image"].to(dev)).argmax(1)[0].to(torch.uint8).cpu().numpy()
            flips += int((pe != g["masks"][i]).sum())
    ref = float(g["f32_dice"])
    nvox = len(val) * int(g["S"]) ** 3
    print(f"\nheld-out Dice on the reference's weights: engine {met['dice']:.7f} vs reference {ref:.7f} "
          f"(|d| {abs(met['dice'] - ref):.2e}); per class {np.round(met['dice_per_class'], 7).tolist()} vs "
          f"{np.round(g['f32_dice_per_class'], 7).tolist()}; val loss {vloss:.8f} vs {float(g['f32_val_loss']):.8f}; "
          f"argmax flips {flips} of {nvox} voxels")
    assert ref > 0.5
    assert abs(met["dice"] - ref) <= 1e-4
    assert np.allclose(met["dice_per_class"], g["f32_dice_per_class"], rtol=0, atol=1e-4)
    assert abs(vloss - float(g["f32_val_loss"])) < 1e-5
    assert flips <= 1e-5 * nvox


def test_heldout_dice_free_running_trained(dev):
    """The same K = 160-step epoch trained BY THE ENGINE from the reference's initial weights (torch.manual_seed
    42 + the reference's registration order), then validated: a free-running trajectory, so the bound is the
    reference's own reproducibility envelope on the same run (envelope(): fp32 at 1/2/4/6/8 threads and fp64,
    0.9334-0.9438 -- the reference at 1 thread lands 9.3e-3 from itself at 8).  Until round 5 the bound was
    max(1e-4, 2 |ref32 - ref64|) around the 8-thread run, which a legitimate fp32 reorder of the engine (round 5's
    runtime-brick routing of the < 128-unit conv shapes, 2dc10ed: 0.93916 -> 0.93402) brought within 13 % of its
    edge; both engine orders sit inside the envelope.  The +-1e-4 north_star check is the pinned-weights test above."""
    g = golden("dice_heldout_trained")
    cfg = _trained_cfg(g)
    torch.manual_seed(42)
    m = build_model(cfg)
    train = [_trained_batch(g, s) for s in g["train_seeds"]]
    val = [_trained_batch(g, s) for s in g["val_seeds"]]
    tr = Trainer(cfg, m, val_loader=val)
    m.train()
    losses = np.array([tr.train_step(b, i) for i, b in enumerate(train)])
    vloss, met = tr._validate()
    ref, ref64 = float(g["f32_dice"]), float(g["f64_dice"])
    spread = abs(ref - ref64)
    lo, hi, vals = envelope("trained", g)
    print(f"\nfree-running 160 steps: engine Dice {met['dice']:.7f}, reference fp32 {ref:.7f}, fp64 {ref64:.7f} "
          f"(|engine - ref| {abs(met['dice'] - ref):.2e}, reference fp32-vs-fp64 spread {spread:.2e}); train loss "
          f"max diff {np.abs(losses - g['f32_train_losses']).max():.2e}; reference envelope (fp32 at 1/2/4/6/8 "
          f"threads, fp64) {np.round(vals, 5).tolist()}; gate [{lo:.5f}, {hi:.5f}], margin "
          f"{min(met['dice'] - lo, hi - met['dice']):.2e}")
    assert lo <= met["dice"] <= hi
