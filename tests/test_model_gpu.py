"""Model-level parity of the HIP engine against the reference, through the
drop-in API (build_model / get_loss / Trainer.train_step):

  * tiny configs: init weights (RNG order), logits, loss, per-parameter grad
    norms and a 3-step AdamW trajectory vs golden fixtures captured from the
    reference (tests/golden/make_golden.py);
  * full BASELINE sizes (UNet3D c2, DualEncoder c3 at 96^3, B=2): logits vs
    the reference's seeded voxel samples, loss, argmax histogram;
  * bf16 storage mode against the same goldens at a bf16 tolerance;
  * bitwise determinism of two identical steps.

Tolerances: fp32 logits 1e-3 normwise relative (north_star), measured ~1e-6.
"""
import copy

import numpy as np
import pytest
import torch

import mmseg_amd  # noqa: F401
from mmseg_amd._lib import lib
from mmseg_amd.models.build import build_model
from mmseg_amd.trainer.losses import get_loss
from mmseg_amd.trainer.trainer import Trainer
from tests.helpers import golden, rel

pytestmark = pytest.mark.gpu


def make_config(model, modalities, out_channels, features, fusion="cross_attention", loss="dice_ce", lr=1e-3,
                dtype="float32", tmp="/tmp/mmseg_test_out"):
    return {
        "experiment": {"name": "t", "output_dir": tmp, "seed": 0},
        "data": {"modalities": list(modalities)},
        "model": {"name": model, "in_channels": len(modalities), "out_channels": out_channels,
                  "backbone": {"features": list(features), "norm": "instance"},
                  "fusion": {"type": fusion}, "head": {"dropout": 0.0}},
        "training": {"epochs": 1, "batch_size": 2, "accumulation_steps": 1,
                     "optimizer": {"name": "adamw", "lr": lr, "weight_decay": 1e-5, "betas": [0.9, 0.999]},
                     "scheduler": {"name": "none"},
                     "loss": {"name": loss, "dice_weight": 0.5, "ce_weight": 0.5, "class_weights": None},
                     "checkpoint": {"save_last": False, "save_best": False}},
        "hardware": {"device": "cuda", "mixed_precision": False, "engine_dtype": dtype},
    }


TINY = {
    "unet_tiny": ("unet", ["CT", "PET"], 3, "cross_attention", "dice_ce"),
    "dual_tiny_cross_attention": ("dual_encoder", ["CT", "PET"], 3, "cross_attention", "dice_ce"),
    "dual_tiny_concat": ("dual_encoder", ["CT", "PET"], 3, "concat", "dice_ce"),
    "dual_tiny_add": ("dual_encoder", ["CT", "PET"], 3, "add", "dice_ce"),
    "dual_tiny_attention": ("dual_encoder", ["CT", "PET"], 3, "attention", "dice_ce"),
    "dual_tiny_m3_tversky": ("dual_encoder", ["CT", "PET", "MRI"], 6, "cross_attention", "tversky"),
}


def _inputs(g, M, C):
    S, B, steps = int(g["S"]), int(g["B"]), int(g["steps"])
    gen = torch.Generator().manual_seed(int(g["seed"]) + 1)
    xs = torch.randn(steps + 1, B, M, S, S, S, generator=gen)
    ys = torch.randint(0, C, (steps + 1, B, S, S, S), generator=gen)
    return xs, ys


def _build(tag, dtype="float32"):
    model, mods, C, fusion, loss = TINY[tag]
    g = golden(tag)
    cfg = make_config(model, mods, C, list(g["features"]), fusion=fusion, loss=loss, dtype=dtype)
    torch.manual_seed(int(g["seed"]))
    m = build_model(cfg)
    return cfg, m, g, len(mods), C


@pytest.mark.parametrize("tag", list(TINY))
def test_tiny_model_matches_reference(dev, tag):
    cfg, m, g, M, C = _build(tag)
    names = list(g["init_names"])
    bb = dict(m.backbone.named_parameters())
    assert list(bb) == names, "parameter registration order differs from the reference"
    init_sum = np.array([bb[n].detach().cpu().double().sum().item() for n in names])
    # double sums are compared to 1e-12: CPU reduction order differs across host CPUs
    assert np.allclose(init_sum, g["init_sum"], rtol=1e-12, atol=1e-12), "initial weights differ (RNG order)"
    xs, ys = _inputs(g, M, C)
    crit = get_loss(cfg)
    m.train()
    out = m(xs[0].to(dev))
    loss = crit(out, ys[0].to(dev))
    loss.backward()
    flat = out.detach().reshape(-1).cpu()
    sidx = torch.from_numpy(g["sample_idx"])
    assert rel(flat[sidx], torch.from_numpy(g["sample_logits"])) < 1e-4
    if "logits" in g:
        assert rel(out, torch.from_numpy(g["logits"])) < 1e-4
    assert abs(loss.item() - float(g["loss"])) < 1e-5
    gn = np.array([bb[n].grad.cpu().double().norm().item() for n in names])
    relg = np.abs(gn - g["grad_norm"]) / np.maximum(g["grad_norm"], 1e-12)
    # conv biases before InstanceNorm have mathematically-zero gradients (fp noise); the
    # transposed-conv bias is nearly dead too (a constant input channel only survives the next IN through
    # the zero-padded border), so its gradient is a heavily cancelling sum: 1e-2 there, 1e-3 elsewhere.
    dead = np.array([n.endswith(("conv1.bias", "conv2.bias")) for n in names])
    near = np.array([n.endswith("up.bias") for n in names])
    assert relg[~dead & ~near].max() < 1e-3, [n for n, r, d in zip(names, relg, dead) if r >= 1e-3 and not d]
    assert relg[near].max() < 1e-2
    assert (gn[dead] < 1e-2 * max(gn[~dead].max(), 1e-12)).all()


@pytest.mark.parametrize("tag", ["unet_tiny", "dual_tiny_cross_attention", "dual_tiny_attention",
                                 "dual_tiny_m3_tversky"])
def test_tiny_trajectory_matches_reference_trainer(dev, tag):
    """3 reference-Trainer AdamW steps at lr 1e-3.  AdamW's first steps move every weight by ~lr*sign(g), so
    weights whose true gradient is ~0 (conv biases in front of InstanceNorm) take +-lr on fp noise in
    BOTH implementations: the trajectory is only loss-level comparable.  Per-step gradient parity is checked
    teacher-forced in test_teacher_forced_steps_match_oracle."""
    cfg, m, g, M, C = _build(tag)
    xs, ys = _inputs(g, M, C)
    tr = Trainer(cfg, m)
    losses = [tr.train_step({"image": xs[1 + i], "label": ys[1 + i]}, i) for i in range(int(g["steps"]))]
    assert np.allclose(losses, g["traj_losses"], rtol=0, atol=1e-4), (losses, g["traj_losses"])
    m.eval()
    with torch.no_grad():
        after = m(xs[0].to(dev)).reshape(-1).cpu()
    assert rel(after[torch.from_numpy(g["sample_idx"])], torch.from_numpy(g["after_sample"])) < 1e-1


def _engine_pins(m, kind):
    """The engine's kink decisions of the forward that just ran (call before the backward, which overwrites the
    pre-norm buffers in place): each block's ReLU masks (pre-norm conv output > its InstanceNorm mean, i.e.
    (x - mean) * rstd > 0, exactly the engine's test) and each MaxPool's argmax codes."""
    from oracle import mmseg_oracle as O
    prog = m.backbone.__dict__["_engine"].program

    def masks(b):
        res = []
        for x, mean in ((b.x1, b.stats[0]), (b.x2, b.stats[2])):
            mu = mean.view(x.N, x.C)[:, :, None, None, None]
            res.append((x.to_ncdhw() > mu).cpu())
        return res

    def codes(idx, l, C):
        D, H, W = prog.dims[l]
        N = prog.shape[0]
        return idx.view(N, D, H, W, C).permute(0, 4, 1, 2, 3).cpu()

    F_ = prog.F
    relu, pool = [], []
    if kind == "unet":
        for b in [prog.init] + prog.enc:
            relu += masks(b)
        pool = [codes(prog.idx[l], l, F_[l - 1]) for l in range(1, prog.L)]
    else:
        for blocks in prog.encs:
            for b in blocks:
                relu += masks(b)
        pool = [codes(prog.idx[mm][l], l, F_[l - 1]) for mm in range(prog.M) for l in range(1, prog.L)]
    for b in prog.dec.blocks:
        relu += masks(b)
    return O.Pins(relu, pool)


@pytest.mark.parametrize("tag", ["unet_tiny", "dual_tiny_attention", "dual_tiny_concat", "dual_tiny_cross_attention",
                                 "dual_tiny_add"])
def test_teacher_forced_steps_pinned_to_oracle(dev, tag):
    """At every step of a GPU training run (fp32) the oracle re-evaluates the step in fp64 from the engine's
    current weights WITH THE ENGINE'S KINK DECISIONS (ReLU masks, MaxPool argmaxes; oracle.Pins): gradients
    then differ by fp32 rounding alone, and every parameter gradient is held to 1e-4 normwise (max|a-b|/max|b|;
    the conv biases in front of an InstanceNorm, whose true gradient is 0, only to the scale of the rest).
    test_teacher_forced_steps_match_oracle below is the free-running form of the same check."""
    from oracle import mmseg_oracle as O
    cfg, m, g, M, C = _build(tag)
    xs, ys = _inputs(g, M, C)
    kind, _, _, fusion, lossname = TINY[tag]
    L = len(g["features"])
    fwd = ((lambda pp, x, pins: O.unet3d_forward(pp, x, L, pins=pins)) if kind == "unet" else
           (lambda pp, x, pins: O.dual_encoder_forward(pp, x, fusion, L, pins=pins)))
    lossf = O.dice_ce_loss if lossname == "dice_ce" else O.tversky_loss
    tr = Trainer(cfg, m)
    for i in range(3):
        m.zero_grad(set_to_none=True)
        m.train()
        out = m(xs[i].to(dev))
        pins = _engine_pins(m, kind)
        loss = tr.criterion(out, ys[i].to(dev))
        loss.backward()
        params = {n: p.detach().cpu().double().requires_grad_(True) for n, p in m.backbone.named_parameters()}
        ro = fwd(params, xs[i].double(), pins)
        rl = lossf(ro, ys[i])
        rl.backward()
        assert pins.ri == len(pins.relu_masks) and pins.pi == len(pins.pool_codes)
        assert rel(out, ro) < 1e-5
        assert abs(loss.item() - rl.item()) < 1e-6
        errs, dead = {}, {}
        for n, p in m.backbone.named_parameters():
            e = rel(p.grad, params[n].grad)
            (dead if n.endswith(("conv1.bias", "conv2.bias")) else errs)[n] = e
        worst = sorted(((v, n) for n, v in errs.items()), reverse=True)[:4]
        print(f"step {i}: pinned grad errors median {np.median(list(errs.values())):.2e}, worst "
              f"{[(float(f'{v:.2e}'), n) for v, n in worst]}")
        assert max(errs.values()) < 1e-4, worst
        gmax = max(float(p.grad.abs().max()) for n, p in m.backbone.named_parameters() if n in errs)
        assert all(float(p.grad.abs().max()) < 1e-2 * gmax for n, p in m.backbone.named_parameters() if n in dead)
        tr.optimizer.step()


@pytest.mark.parametrize("tag", ["unet_tiny", "dual_tiny_attention", "dual_tiny_concat", "dual_tiny_cross_attention"])
def test_teacher_forced_steps_match_oracle(dev, tag):
    """At every step of a GPU training run the oracle re-evaluates loss and gradients from the GPU's current
    weights in fp32 and in fp64.  fp32 itself is not exact here: a pre-activation within rounding of 0 flips its
    ReLU mask and a MaxPool near-tie flips its argmax, and either reroutes one voxel's gradient discretely; a
    flip near the head perturbs EVERY gradient by ~1e-3 (tools/diag_tf.py: the fp32 oracle shows 3e-4 at one
    step and 2e-6 at the next, the engine hits its flips at other steps).  A flip is a rounding-order event,
    so the bound is not "as close as the fp32 oracle at this step" but the size such events reach: every
    gradient within max(10x the fp32 oracle's error, 0.25) normwise (near-dead gradients, 1e-3 of the typical
    per-element scale, are skipped), and the median over parameters within 3e-2.  A wiring error (wrong buffer,
    missing term, stale weights) moves a gradient by O(1); flips measured here reach ~0.1 on single layers.
    Bit-level agreement of every kernel is covered by tests/test_kernels_gpu.py."""
    from oracle import mmseg_oracle as O
    cfg, m, g, M, C = _build(tag)
    xs, ys = _inputs(g, M, C)
    kind, _, _, fusion, lossname = TINY[tag]
    fwd = O.unet3d_forward if kind == "unet" else (lambda pp, x: O.dual_encoder_forward(pp, x, fusion))
    lossf = O.dice_ce_loss if lossname == "dice_ce" else O.tversky_loss
    tr = Trainer(cfg, m)
    for i in range(3):
        refs = {}
        for dt in (torch.float32, torch.float64):
            params = {n: p.detach().cpu().to(dt).requires_grad_(True) for n, p in m.backbone.named_parameters()}
            ro = fwd(params, xs[i].to(dt))
            rl = lossf(ro, ys[i])
            rl.backward()
            refs[dt] = (ro, rl, params)
        out = m(xs[i].to(dev))
        loss = tr.criterion(out, ys[i].to(dev))
        m.zero_grad(set_to_none=True)
        loss.backward()
        r32, r64 = refs[torch.float32], refs[torch.float64]
        assert rel(out, r64[0]) < 1e-4
        assert abs(loss.item() - r64[1].item()) < 1e-5
        e_eng, e_ref, scale = {}, {}, {}
        for n, p in m.backbone.named_parameters():
            if n.endswith(("conv1.bias", "conv2.bias")):
                continue  # mathematically zero (bias in front of InstanceNorm)
            g64 = r64[2][n].grad
            e_eng[n] = rel(p.grad, g64)
            e_ref[n] = rel(r32[2][n].grad, g64)
            scale[n] = float(g64.norm()) / g64.numel() ** 0.5
        typical = float(np.median(list(scale.values())))
        bad = {n: (e_eng[n], e_ref[n]) for n in e_eng
               if scale[n] > 1e-3 * typical and e_eng[n] > max(10 * e_ref[n], 0.25)}
        assert not bad, (i, bad)
        med_eng = float(np.median(list(e_eng.values())))
        print(f"step {i}: median engine grad error {med_eng:.3e}; largest:",
              sorted(((round(v, 4), n) for n, v in e_eng.items()), reverse=True)[:6])
        # a flip at one ReLU / pooling decision spreads over every layer below it: unet_tiny step 1 measured a
        # 1.07e-2 median after the head weight-gradient reduction order changed (other steps 2e-6, other
        # models <= 4e-3 at their flip steps); a wiring error is O(1)
        assert med_eng < 3e-2, (i, med_eng, float(np.median(list(e_ref.values()))))
        tr.optimizer.step()


@pytest.mark.parametrize("tag", ["unet_tiny", "dual_tiny_cross_attention"])
def test_tiny_bf16_close_to_reference(dev, tag):
    cfg, m, g, M, C = _build(tag, dtype="bfloat16")
    xs, ys = _inputs(g, M, C)
    out = m(xs[0].to(dev))
    flat = out.detach().reshape(-1).cpu()
    assert rel(flat[torch.from_numpy(g["sample_idx"])], torch.from_numpy(g["sample_logits"])) < 5e-2
    assert abs(get_loss(cfg)(out, ys[0].to(dev)).item() - float(g["loss"])) < 5e-3


def test_step_bitwise_deterministic(dev):
    cfg, m, g, M, C = _build("dual_tiny_attention")
    xs, ys = _inputs(g, M, C)
    crit = get_loss(cfg)
    grads = []
    for _ in range(2):
        m.zero_grad(set_to_none=True)
        crit(m(xs[0].to(dev)), ys[0].to(dev)).backward()
        grads.append(torch.cat([p.grad.reshape(-1).clone() for p in m.parameters()]))
    assert torch.equal(grads[0], grads[1])


@pytest.mark.parametrize("tag", ["dual_tiny_cross_attention", "dual_tiny_m3_tversky"])
def test_modality_streams_bitwise_equal(dev, tag, monkeypatch):
    """The optional per-modality HIP streams (MMSEG_MODALITY_STREAMS=1) run the same kernels in the same
    per-modality order: logits and every gradient must be bitwise those of the single-stream step."""
    cfg, m, g, M, C = _build(tag)
    xs, ys = _inputs(g, M, C)
    crit = get_loss(cfg)
    res = []
    for streams in ("0", "1"):
        monkeypatch.setenv("MMSEG_MODALITY_STREAMS", streams)
        m.zero_grad(set_to_none=True)
        out = m(xs[0].to(dev))
        crit(out, ys[0].to(dev)).backward()
        torch.cuda.synchronize()
        res.append((out.detach().clone(), torch.cat([p.grad.reshape(-1).clone() for p in m.parameters()])))
    assert torch.equal(res[0][0], res[1][0])
    assert torch.equal(res[0][1], res[1][1])


def test_accumulation_matches_two_batch_sum(dev):
    """accumulation_steps=2 must equal the average of the two micro-batch gradients."""
    cfg, m, g, M, C = _build("unet_tiny")
    xs, ys = _inputs(g, M, C)
    crit = get_loss(cfg)
    m2 = copy.deepcopy(m)
    m.zero_grad(set_to_none=True)
    (crit(m(xs[0].to(dev)), ys[0].to(dev)) / 2).backward()
    (crit(m(xs[1].to(dev)), ys[1].to(dev)) / 2).backward()
    acc = torch.cat([p.grad.reshape(-1) for p in m.parameters()]).clone()
    parts = []
    for i in range(2):
        m2.zero_grad(set_to_none=True)
        crit(m2(xs[i].to(dev)), ys[i].to(dev)).backward()
        parts.append(torch.cat([p.grad.reshape(-1) for p in m2.parameters()]).clone())
    assert rel(acc, (parts[0] + parts[1]) / 2) < 1e-5


def test_validate_dice(dev):
    cfg, m, g, M, C = _build("unet_tiny")
    xs, ys = _inputs(g, M, C)
    tr = Trainer(cfg, m, val_loader=[{"image": xs[i], "label": ys[i]} for i in range(2)])
    vloss, met = tr._validate()
    assert 0.0 <= met["dice"] <= 1.0 and len(met["dice_per_class"]) == C and np.isfinite(vloss)


@pytest.mark.parametrize("tag,model", [("full_unet_c2", "unet"), ("full_dual_c3", "dual_encoder")])
def test_full_size_forward_matches_reference(dev, tag, model):
    g = golden(tag)
    S, B, seed = int(g["S"]), int(g["B"]), int(g["seed"])
    cfg = make_config(model, ["CT", "PET"], 6, [32, 64, 128, 256, 512])
    torch.manual_seed(seed)
    m = build_model(cfg)
    psum = np.array([p.detach().cpu().double().sum().item() for p in m.backbone.parameters()])
    assert np.allclose(psum, g["param_sum"], rtol=1e-12, atol=1e-12)
    rng = np.random.Generator(np.random.PCG64(seed + 100))
    x = torch.from_numpy(rng.standard_normal((B, 2, S, S, S), dtype=np.float32))
    y = torch.from_numpy(rng.integers(0, 6, size=(B, S, S, S)).astype(np.int64))
    idx = torch.from_numpy(rng.integers(0, S ** 3, size=1024))
    assert torch.equal(idx, torch.from_numpy(g["sample_idx"]))
    m.eval()
    with torch.no_grad():
        out = m(x.to(dev))
        loss = get_loss(cfg)(out, y.to(dev))
    samp = out.reshape(B, 6, -1)[:, :, idx.to(dev)].cpu()
    assert rel(samp, torch.from_numpy(g["sample_logits"])) < 1e-3
    assert abs(loss.item() - float(g["loss"])) < 1e-4 * abs(float(g["loss"]))
    hist = torch.bincount(out.argmax(1).reshape(-1), minlength=6).cpu().numpy()
    assert np.abs(hist - g["argmax_hist"]).sum() <= 1e-4 * hist.sum()


@pytest.mark.parametrize("fused", ["1", "0"])
def test_train_step_raises_on_out_of_range_labels(dev, fused, monkeypatch):
    """reference: F.one_hot raises on a class index >= num_classes BEFORE any update; Trainer.train_step raises
    too, and the model is untouched: the loss kernels count such voxels on the device, the AdamW kernel skips
    its update when that count is non-zero (no host sync), the step counter is rolled back, and the next good
    step gives bitwise the state of a run that never saw the bad batch (fused head + loss and unfused)."""
    monkeypatch.setenv("MMSEG_FUSED_HEAD_LOSS", fused)
    xs = None
    runs = []
    for with_bad in (True, False):
        cfg, m, g, M, C = _build("unet_tiny")
        xs, ys = _inputs(g, M, C)
        tr = Trainer(cfg, m)
        tr.train_step({"image": xs[0], "label": ys[0]}, 0)
        if with_bad:
            before = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).clone()
            mom = [t.clone() for t in tr.optimizer._flat[0]]
            bad = ys[1].clone()
            bad[0, 0, 0, 0] = C
            with pytest.raises(RuntimeError, match="outside"):
                tr.train_step({"image": xs[1], "label": bad}, 1)
            after = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
            assert torch.equal(before, after), "a bad batch updated the parameters"
            assert all(torch.equal(a, b) for a, b in zip(mom, tr.optimizer._flat[0])), "moments changed"
            assert int(tr.optimizer.state[next(m.parameters())]["step"]) == 1
        tr.train_step({"image": xs[2], "label": ys[2]}, 2)
        runs.append(torch.cat([p.detach().reshape(-1) for p in m.parameters()]).clone())
    assert torch.equal(runs[0], runs[1])


def test_focal_ignores_minus_100(dev):
    """FocalLoss (reference losses.py:83-125): F.cross_entropy(reduction='none') gives 0 at torch's default
    ignore_index -100 and .mean() still counts those voxels; the HIP kernels do the same (loss and gradient vs
    the reference formula evaluated by torch on the CPU in fp64).  No NaN, nothing raised."""
    import torch.nn.functional as F
    from mmseg_amd.trainer.losses import FocalLoss
    g = torch.Generator().manual_seed(21)
    for C in (3, 6):
        logits = torch.randn(2, C, 6, 7, 8, generator=g) * 3
        y = torch.randint(0, C, (2, 6, 7, 8), generator=g)
        y[torch.rand(y.shape, generator=g) < 0.2] = -100
        cw = torch.rand(C, generator=g) + 0.5
        for alpha in (None, cw):
            ref_in = logits.double().requires_grad_(True)
            ce = F.cross_entropy(ref_in, y, weight=None if alpha is None else alpha.double(), reduction="none")
            pt = torch.exp(-ce)
            ref = ((1 - pt) ** 2.0 * ce).mean()
            ref.backward()
            x = logits.to(dev).requires_grad_(True)
            loss = FocalLoss(alpha=alpha)(x, y.to(dev))
            loss.backward()
            assert abs(loss.item() - ref.item()) < 1e-5 * max(1.0, abs(ref.item())), (C, loss.item(), ref.item())
            assert rel(x.grad.cpu(), ref_in.grad) < 1e-5


@pytest.mark.parametrize("dropout", [0.3, 0.0])
@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
@pytest.mark.parametrize("tag", ["unet_tiny", "dual_tiny_cross_attention"])
def test_fused_head_loss_matches_unfused(dev, tag, dtype, dropout):
    """Trainer's fused head + loss node (engine.run_engine_loss: no logits / dlogits tensors, logits recomputed
    in the backward) against model(x) -> criterion -> backward, for every HIP loss, class weights, uint8 labels,
    with an active Dropout3d (same device RNG state for both runs) and without one -- in bf16 the fused kernels'
    logits then come from the bf16 hi + lo MFMAs (MMSEG_HEAD_BF16, loss_head.hip head_logits_bf)."""
    from mmseg_amd.engine.engine import fused_loss_supported, run_engine_loss
    from mmseg_amd.trainer.losses import CrossEntropyLoss, DiceCELoss, DiceLoss, FocalLoss, TverskyLoss
    cfg, m, g, M, C = _build(tag, dtype)
    m.backbone.dropout_p = dropout
    m.train()
    xs, ys = _inputs(g, M, C)
    x, y = xs[0].to(dev), ys[0].to(dev)
    bb = m.backbone
    kind = "unet" if tag == "unet_tiny" else "dual_encoder"
    assert fused_loss_supported(bb, kind, x)
    cw = torch.rand(C, generator=torch.Generator().manual_seed(3)) + 0.5
    losses = {"dicece": DiceCELoss(), "dicece_w": DiceCELoss(0.3, 0.7, class_weights=cw), "dice": DiceLoss(),
              "ce_w": CrossEntropyLoss(weight=cw), "tversky": TverskyLoss(0.3, 0.7), "focal": FocalLoss()}
    tol = 1e-5 if dtype == "float32" else 2e-2
    for name, crit in losses.items():
        for lab in (y, y.to(torch.uint8)):
            res = []
            for fused in (False, True):
                m.zero_grad(set_to_none=True)
                torch.cuda.manual_seed(7)
                if fused:
                    c = getattr(crit, "class_weights", None)
                    c = None if c is None else c.to(dev, torch.float32)
                    loss = run_engine_loss(bb, kind, x, lab, crit._spec(), c)
                else:
                    loss = crit(m(x), lab)
                (loss * 0.5).backward()
                torch.cuda.synchronize()
                # conv biases in front of an InstanceNorm have a gradient of pure rounding noise (DESIGN (a)):
                # compared are the weights and the head's bias
                res.append((loss.item(), [p.grad.detach().double().cpu().clone() for n, p in m.named_parameters()
                                          if not n.endswith("bias") or "out_conv" in n]))
            (lu, gu), (lf, gf) = res
            assert abs(lu - lf) <= 1e-5 * max(1.0, abs(lu)), (name, lu, lf)
            for a, b in zip(gf, gu):
                assert ((a - b).norm() / b.norm()).item() < tol, (name, dtype)


@pytest.mark.parametrize("tag", ["unet_tiny", "dual_tiny_cross_attention"])
def test_head_bf16_logits_match_fp32_logits(dev, tag, monkeypatch):
    """bf16 storage, no Dropout3d: the fused head + loss kernels' logits from bf16 hi + lo MFMAs (x exact in bf16,
    W to ~2^-17) against the exact fp32 MFMA chain (MMSEG_HEAD_BF16=0): loss to 1e-5, gradients to the bf16
    fused-vs-unfused bound (2e-2: a logit change of ~1e-6 can move a bf16 rounding downstream)."""
    from mmseg_amd.engine.engine import fused_loss_supported, run_engine_loss
    from mmseg_amd.trainer.losses import DiceCELoss, TverskyLoss
    cfg, m, g, M, C = _build(tag, "bfloat16")
    m.backbone.dropout_p = 0.0
    m.train()
    xs, ys = _inputs(g, M, C)
    x, y = xs[0].to(dev), ys[0].to(dev)
    kind = "unet" if tag == "unet_tiny" else "dual_encoder"
    assert fused_loss_supported(m.backbone, kind, x)
    for crit in (DiceCELoss(), TverskyLoss(0.3, 0.7)):
        res = []
        for bf in ("0", "1"):
            monkeypatch.setenv("MMSEG_HEAD_BF16", bf)
            m.zero_grad(set_to_none=True)
            loss = run_engine_loss(m.backbone, kind, x, y, crit._spec(), None)
            loss.backward()
            torch.cuda.synchronize()
            res.append((loss.item(), [p.grad.detach().double().cpu().clone() for n, p in m.named_parameters()
                                      if not n.endswith("bias") or "out_conv" in n]))
        (l0, g0), (l1, g1) = res
        assert abs(l0 - l1) <= 1e-5 * max(1.0, abs(l0)), (l0, l1)
        worst = max(((a - b).norm() / max(b.norm(), 1e-30)).item() for a, b in zip(g1, g0))
        print(f"{tag} {type(crit).__name__}: loss {l0:.7f} vs {l1:.7f}, worst gradient rel {worst:.2e}")
        assert worst < 2e-2


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
@pytest.mark.parametrize("tag", ["unet_tiny", "dual_tiny_cross_attention"])
def test_deferred_head_norm_bitwise(dev, tag, dtype, monkeypatch):
    """Fused head + loss: the last decoder block's InstanceNorm + ReLU applied on load by the head kernels (its
    output never written) gives a bit-identical loss and gradients to the materialised path
    (MMSEG_DEFER_HEAD_NORM=0), with an active Dropout3d."""
    from mmseg_amd.engine.engine import fused_loss_supported, run_engine_loss
    from mmseg_amd.trainer.losses import DiceCELoss
    kind = "unet" if tag == "unet_tiny" else "dual_encoder"
    res = []
    for defer in ("1", "0"):
        monkeypatch.setenv("MMSEG_DEFER_HEAD_NORM", defer)
        cfg, m, g, M, C = _build(tag, dtype)
        m.backbone.dropout_p = 0.3
        m.train()
        xs, ys = _inputs(g, M, C)
        assert fused_loss_supported(m.backbone, kind, xs[0].to(dev))
        torch.cuda.manual_seed(7)
        loss = run_engine_loss(m.backbone, kind, xs[0].to(dev), ys[0].to(dev), DiceCELoss()._spec(), None)
        loss.backward()
        torch.cuda.synchronize()
        assert m.backbone.__dict__["_engine"].program.dec.blocks[-1].defer_out == (defer == "1")
        res.append((loss.detach().clone(), torch.cat([p.grad.reshape(-1) for p in m.parameters()]).clone()))
    assert torch.equal(res[0][0], res[1][0])
    assert torch.equal(res[0][1], res[1][1])


@pytest.mark.parametrize("wgrad_dma", ["0", "1"])
@pytest.mark.parametrize("model", ["unet", "dual_encoder"])
def test_deferred_conv_norm_bitwise(dev, model, wgrad_dma, monkeypatch):
    """bf16, 32-channel top level (the brick6 forward and the wgrad_row weight gradient at W = 32): conv1's
    InstanceNorm + ReLU applied by conv2's forward and weight-gradient kernels on staging (y1 never written) gives a
    bit-identical loss and gradients to the materialised path (MMSEG_DEFER_CONV_NORM=0)."""
    from mmseg_amd.engine.engine import fused_loss_supported, run_engine_loss
    from mmseg_amd.trainer.losses import DiceCELoss
    gen = torch.Generator().manual_seed(5)
    x = torch.randn(2, 2, 32, 32, 32, generator=gen).to(dev)
    y = torch.randint(0, 3, (2, 32, 32, 32), generator=gen).to(dev)
    res = []
    # register-staged / LDS-DMA weight-gradient kernels, the same kind on both paths (their bias gradients sum
    # in different orders)
    monkeypatch.setenv("MMSEG_WGRAD_DMA", wgrad_dma)
    for defer in ("1", "0"):
        monkeypatch.setenv("MMSEG_DEFER_CONV_NORM", defer)
        cfg = make_config(model, ["CT", "PET"], 3, [32, 64, 128], dtype="bfloat16")
        torch.manual_seed(0)
        m = build_model(cfg).to(dev)
        m.train()
        assert fused_loss_supported(m.backbone, model, x)
        loss = run_engine_loss(m.backbone, model, x, y, DiceCELoss()._spec(), None)
        loss.backward()
        torch.cuda.synchronize()
        prog = m.backbone.__dict__["_engine"].program
        top = prog.init if model == "unet" else prog.encs[0][0]
        assert top.defer1 == (defer == "1") and prog.dec.blocks[-1].defer1 == (defer == "1")
        res.append((loss.detach().clone(), torch.cat([p.grad.reshape(-1) for p in m.parameters()]).clone()))
    assert torch.equal(res[0][0], res[1][0])
    assert torch.equal(res[0][1], res[1][1])


@pytest.mark.parametrize("knob,defer_head", [("MMSEG_HEAD_IN_PART", "1"), ("MMSEG_HEAD_IN_PART", "0"),
                                             ("MMSEG_DGRAD_IN_PART", "1")])
@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
@pytest.mark.parametrize("model", ["unet", "dual_encoder"])
def test_head_in_partials(dev, model, dtype, knob, defer_head, monkeypatch):
    """32-channel top level: InstanceNorm-backward partial sums emitted by the producer of dy instead of a partial
    pass over x and dy -- by the fused head + loss backward for the last decoder block's output norm
    (MMSEG_HEAD_IN_PART, mmseg_head_loss_bwd_in) and by conv2's brick5 data gradient for conv1's norm in every
    96^3-style block (MMSEG_DGRAD_IN_PART, mmseg_conv3_dgrad_in, bf16 only); both feed mmseg_instnorm_bwd_part.
    Same loss bits; gradients equal to the two-pass path (knob=0) up to the summation order of those partials
    (fp32 1e-5, bf16 1e-2 normwise: a bf16 activation rounding on the other side moves by one ulp); the head's own
    weight gradient is untouched (bitwise)."""
    from mmseg_amd.engine.engine import fused_loss_supported, run_engine_loss
    from mmseg_amd.trainer.losses import DiceCELoss
    gen = torch.Generator().manual_seed(9)
    x = torch.randn(2, 2, 32, 32, 32, generator=gen).to(dev)
    y = torch.randint(0, 3, (2, 32, 32, 32), generator=gen).to(dev)
    monkeypatch.setenv("MMSEG_DEFER_HEAD_NORM", defer_head)
    res = []
    for fused in ("1", "0"):
        monkeypatch.setenv(knob, fused)
        cfg = make_config(model, ["CT", "PET"], 3, [32, 64, 128], dtype=dtype)
        torch.manual_seed(0)
        m = build_model(cfg).to(dev)
        m.train()
        assert fused_loss_supported(m.backbone, model, x)
        loss = run_engine_loss(m.backbone, model, x, y, DiceCELoss()._spec(), None)
        loss.backward()
        torch.cuda.synchronize()
        prog = m.backbone.__dict__["_engine"].program
        if knob == "MMSEG_HEAD_IN_PART":
            assert (getattr(prog.dec, "_hpart", None) is not None) == (fused == "1")
        else:
            assert (getattr(prog.dec.blocks[-1].c2, "_inpart", None) is not None) == (fused == "1" and
                                                                                   dtype == "bfloat16")
        head = [p.grad.reshape(-1).clone() for n, p in m.named_parameters() if "out_conv" in n]
        res.append((loss.detach().clone(), torch.cat([p.grad.reshape(-1) for p in m.parameters()]).clone(), head))
    assert torch.equal(res[0][0], res[1][0])
    for a, b in zip(res[0][2], res[1][2]):
        assert torch.equal(a, b)
    a, b = res[0][1].double(), res[1][1].double()
    err = ((a - b).norm() / b.norm()).item()
    assert err < (1e-5 if dtype == "float32" else 1e-2), err


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
@pytest.mark.parametrize("model", ["unet", "dual_encoder"])
def test_stem_inb_engaged(dev, model, dtype):
    """The top block's conv1 is the stem: its InstanceNorm backward is applied by the stem weight gradient while it
    stages dy (mmseg_instnorm_bwd_coef + mmseg_stem_wgrad_inb, the norm's input gradient never written).  Here: it
    engages at 32^3 and yields finite gradients; its values are held to the reference by the golden whole-model and
    full-size pinned tests, which run it (its materialised A/B switch measured bitwise equal, r04, and was removed
    in round 6)."""
    from mmseg_amd.engine.engine import fused_loss_supported, run_engine_loss
    from mmseg_amd.trainer.losses import DiceCELoss
    gen = torch.Generator().manual_seed(11)
    x = torch.randn(2, 2, 32, 32, 32, generator=gen).to(dev)
    y = torch.randint(0, 3, (2, 32, 32, 32), generator=gen).to(dev)
    cfg = make_config(model, ["CT", "PET"], 3, [32, 64, 128], dtype=dtype)
    torch.manual_seed(0)
    m = build_model(cfg).to(dev)
    m.train()
    assert fused_loss_supported(m.backbone, model, x)
    loss = run_engine_loss(m.backbone, model, x, y, DiceCELoss()._spec(), None)
    loss.backward()
    torch.cuda.synchronize()
    prog = m.backbone.__dict__["_engine"].program
    top = prog.init if model == "unet" else prog.encs[0][0]
    assert getattr(top, "_coef", None) is not None
    g = torch.cat([p.grad.reshape(-1) for p in m.parameters()])
    assert torch.isfinite(g).all() and torch.isfinite(loss)


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_deferred_encoder_norm_bitwise(dev, dtype, monkeypatch):
    """DualEncoder mean fusion: the encoders' output InstanceNorm + ReLU applied on load by the maxpool and the
    fusion kernel (never written) gives bit-identical logits, gradients and return_features to the
    materialised path (MMSEG_DEFER_ENC_NORM=0)."""
    g = golden("dual_tiny_cross_attention")
    res = []
    for defer in ("1", "0"):
        monkeypatch.setenv("MMSEG_DEFER_ENC_NORM", defer)
        cfg, m, g, M, C = _build("dual_tiny_cross_attention", dtype)
        xs, ys = _inputs(g, M, C)
        crit = get_loss(cfg)
        out = m(xs[0].to(dev))
        crit(out, ys[0].to(dev)).backward()
        _, feats = m(xs[0].to(dev), return_features=True)
        assert m.backbone.__dict__["_engine"].program.encs[0][0].defer_out == (defer == "1")
        res.append((out.detach().clone(), torch.cat([p.grad.reshape(-1) for p in m.parameters()]).clone(),
                    [f.clone() for lvl in feats["encoder_features"] for f in lvl]))
    assert torch.equal(res[0][0], res[1][0])
    assert torch.equal(res[0][1], res[1][1])
    assert all(torch.equal(a, b) for a, b in zip(res[0][2], res[1][2]))


@pytest.mark.parametrize("dtype", ["bfloat16", "float32"])
def test_batched_weight_gradient_reduce_bitwise(dev, dtype, monkeypatch):
    """MMSEG_WRED_BATCH=1 queues every 3^3 weight-gradient split reduce of the backward and sums them in one launch
    at its end (wgrad_reduce_batch_kernel): each gradient is summed over the same splits in the same order as its
    own reduce, so the whole step's gradients are BITWISE the unbatched ones; the queue is empty afterwards."""
    kind, mods, C, fusion, lossname = TINY["dual_tiny_cross_attention"]
    g = golden("dual_tiny_cross_attention")
    gen = torch.Generator().manual_seed(3)
    x = torch.randn(2, len(mods), 96, 96, 96, generator=gen)
    y = torch.randint(0, C, (2, 96, 96, 96), generator=gen)
    res = {}
    for flag in ("0", "1"):
        monkeypatch.setenv("MMSEG_WRED_BATCH", flag)
        cfg = make_config(kind, mods, C, list(g["features"]), fusion=fusion, loss=lossname, dtype=dtype)
        torch.manual_seed(int(g["seed"]))
        m = build_model(cfg)
        tr = Trainer(cfg, m)
        m.train()
        loss = tr.criterion(m(x.to(dev)), y.to(dev))
        loss.backward()
        torch.cuda.synchronize()
        res[flag] = (loss.item(), {n: p.grad.detach().clone() for n, p in m.backbone.named_parameters()})
        assert lib().mmseg_wgrad_reduce_pending() == 0
    assert res["0"][0] == res["1"][0]
    diff = [n for n in res["0"][1] if not torch.equal(res["0"][1][n], res["1"][1][n])]
    assert not diff, diff


@pytest.mark.parametrize("tag,force", [("dual_tiny_cross_attention", "0"), ("dual_tiny_add", "0"),
                                       ("dual_tiny_m3_tversky", "0"), ("dual_tiny_cross_attention", "1"),
                                       ("dual_tiny_m3_tversky", "1"), ("dual_tiny_cross_attention", "w")])
def test_grouped_modalities_match_per_modality(dev, tag, force, monkeypatch):
    """bf16 (the dtype whose small levels take the runtime-brick kernels): the modality-grouped small levels and the
    grouped encoder output-norm backward (MMSEG_GROUP_SMALL, programs.DualEncoderProgram)
    against the per-modality launches on the same weights and batch.  The grouped launches split the reductions
    differently (one launch over M x N samples), so the two differ by bf16 rounding: loss within 1e-3 relative,
    logits within 2e-2 and every gradient within 5e-2 normwise (L2).  force=1 (MMSEG_GROUP_FORCE_R): the 24^3
    level is grouped too, on the runtime-brick kernels instead of the (4, 8, 8)-brick family."""
    monkeypatch.setenv("MMSEG_GROUP_FORCE_R", "1" if force == "1" else "0")
    kind, mods, C, fusion, lossname = TINY[tag]
    g = golden(tag)
    # 96^3 (B = 1, the tiny features): levels 12^3 / 6^3 take the runtime-brick kernels, as in the bench
    gen = torch.Generator().manual_seed(11)
    B = 1
    x = torch.randn(B, len(mods), 96, 96, 96, generator=gen)
    y = torch.randint(0, C, (B, 96, 96, 96), generator=gen)
    res = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("MMSEG_GROUP_SMALL", flag)       # (grouped small levels and grouped output norm)
        # (force: features whose 24^3 convs have unpadded channels -- the tiny fixture's 16 -> 32 conv pads its
        # input channels, which keeps that level per modality)
        feats = [16, 32, 64, 128, 256] if force in ("1", "w") else list(g["features"])
        cfg = make_config(kind, mods, C, feats, fusion=fusion, loss=lossname, dtype="bfloat16")
        torch.manual_seed(int(g["seed"]))
        m = build_model(cfg)
        tr = Trainer(cfg, m)
        m.train()
        loss = tr.criterion(m(x.to(dev)), y.to(dev))
        loss.backward()
        prog = m.backbone.__dict__["_engine"].program
        with torch.no_grad():
            logits = m(x.to(dev)).float().cpu()
        res[flag] = (loss.item(), logits, {n: p.grad.detach().double().cpu().clone()
                                           for n, p in m.backbone.named_parameters()}, prog.l0, prog.L,
                     prog.group_outnorm)
    (l1, lg1, g1, l0, L, go), (l2, lg2, g2, l0b, _, gob) = res["1"], res["0"]
    print(f"\n{tag}: grouped from level {l0} of {L} (output norm grouped: {go}); loss {l1:.6f} vs {l2:.6f}")
    assert l0 == (2 if force == "1" else 3) and go and l0b == L and not gob
    bad_all = {n: float((g1[n] - g2[n]).norm() / g2[n].norm()) for n in g2 if g2[n].norm() > 0}
    print("largest gradient differences:", sorted(bad_all.items(), key=lambda kv: -kv[1])[:6])
    assert abs(l1 - l2) < 1e-3 * abs(l2)
    assert float((lg1 - lg2).norm() / lg2.norm()) < 2e-2
    if force == "1":
        # the forced 24^3 level runs other kernels (runtime-brick) than the per-modality step, so the two bf16
        # steps differ by rounding amplified through kink flips (up to ~0.15 on these random-input gradients, the
        # size of any two bf16 kernel paths here); its parity is held to the pinned fp64 oracle instead
        # (test_fullsize_step_pinned_to_fp64_oracle, group "force")
        return
    bad = {n: float((g1[n] - g2[n]).norm() / g2[n].norm()) for n in g2
           if not n.endswith(("conv1.bias", "conv2.bias")) and g2[n].norm() > 0
           and float((g1[n] - g2[n]).norm() / g2[n].norm()) > 5e-2}
    assert not bad, bad


def test_unet_features48_first_conv_not_the_stem(dev):
    """A UNet3D whose first conv has 48 outputs AND a bias (features[0] = 48, reference unet.py:26) is not the
    bias-free SwinUNETR 48-channel stem (advisor r05): Conv3._stem refuses it (the stem weight gradient has no bias
    term, no fused statistics and no fused norm backward).  Such a UNet / DualEncoder is outside the engine's
    channel contract anyway (8 x 2^k channels per activation, runtime.py; no BASELINE config uses 48): building
    its program raises a clean ValueError instead of reaching a kernel."""
    feats = [48, 96, 192]
    cfg = make_config("unet", ["CT", "PET"], 3, feats)
    torch.manual_seed(0)
    m = build_model(cfg).to(dev)
    x = torch.randn(1, 2, 32, 32, 32, device=dev)
    with pytest.raises(ValueError, match="8 x a power of two"):
        m(x)
    from mmseg_amd.engine.layers import Conv3
    c = Conv3.__new__(Conv3)
    c.Co, c.conv = 48, m.backbone.init_conv.conv1
    assert c.conv.bias is not None and not c._stem(None, 0)
