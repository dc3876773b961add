"""Full-size training-step parity: the engine's step at the BASELINE sizes (96^3, B=2) against the reference's
own training step captured by tests/golden/make_golden.py (full_grad_case: reference train-mode forward + loss +
backward, trainer.py:250-254), run three ways on the CPU: as is (fp32), in fp64 (the rounding-free answer) and
under torch.autocast("cpu", bfloat16) (the CPU analogue of the reference's own mixed-precision step,
trainer.py:237-243).

Cases: c2 UNet3D CT+PET 6 classes DiceCE; c3 DualEncoder "cross_attention" (= mean fusion, the bench
workload) DiceCE; c5 DualEncoder CT+PET+MRI Tversky.  Each runs in fp32 (the parity path) and in bf16 (the path
bench.py times: brick5 / brick3 / brick2-BN64 with 32-bit staging, wgrad_dma, the fused InstanceNorm partials,
the fused head + loss), through Trainer._fused_loss exactly as Trainer.train_step does.

Why the gradient bounds are relative to the reference's own rounding error: at 96^3 every weight gradient is a
heavily cancelling sum over 1.8 M voxels, and a ReLU / MaxPool decision within rounding of its kink routes one
voxel's gradient discretely.  The reference's OWN fp32 gradients differ from its fp64 ones by 3e-3..8e-3
(median over tensors), its bf16-autocast gradients by 0.43..0.50 -- on these random inputs the gradient is
mostly noise that rounding re-draws.  So per parameter tensor (normwise L2 on the fixture's 4096 seeded
positions, all of them for smaller tensors), with e(x) = ||x - ref_fp64|| / ||ref_fp64||:
  * fp32 engine: e(engine) <= max(4 e(ref_fp32), 2 median e(ref_fp32)), and median e(engine) <= 2 median
    e(ref_fp32);
  * bf16 engine: e(engine) <= max(2 e(ref_bf16), median e(ref_bf16)), and median e(engine) <= 1.5 median
    e(ref_bf16).
A wiring error (a wrong buffer, a missing term) moves a gradient by O(1) and its norm by O(1); the gradient
norms are held to 1e-3 (fp32) / 5e-2 (bf16) of the reference's.  Conv biases in front of an InstanceNorm
have a mathematically zero gradient (rounding noise): bounded by 10x the reference's own noise there.
Loss: fp32 1e-5 relative to fp64; bf16 1e-3.  Sampled logits: 1e-3 normwise (north_star) / 3e-2 (bf16).
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


def _l2(a, b):
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


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
    bf = dtype == "bfloat16"
    loss64 = float(g["loss64"])
    err_loss = abs(lossv.item() - loss64) / abs(loss64)
    err_logits = rel(logits.reshape(B, C, -1)[:, :, torch.from_numpy(idx).to(dev)],
                     torch.from_numpy(g["sample_logits64"]))
    bb = dict(m.backbone.named_parameters())
    off = g["gs_off"]
    ref_key = "gs_valbf" if bf else "gs_val"
    e_eng, e_ref, norm_err, dead = {}, {}, {}, {}
    for i, n in enumerate(names):
        sl = slice(off[i], off[i + 1])
        gi = torch.from_numpy(g["gs_idx"][sl]).to(dev)
        g64 = g["gs_val64"][sl]
        geng = bb[n].grad.reshape(-1)[gi].double().cpu().numpy()
        if n.endswith(("conv1.bias", "conv2.bias")):
            dead[n] = (float(np.linalg.norm(geng)), float(np.linalg.norm(g[ref_key][sl])))
            continue
        e_eng[n] = _l2(geng, g64)
        e_ref[n] = _l2(g[ref_key][sl], g64)
        norm_err[n] = abs(float(bb[n].grad.double().norm()) - float(g["grad_norm64"][i])) / float(g["grad_norm64"][i])
    med_eng, med_ref = float(np.median(list(e_eng.values()))), float(np.median(list(e_ref.values())))
    ratio = {n: e_eng[n] / e_ref[n] for n in e_eng}
    worst = sorted(((r, n) for n, r in ratio.items()), reverse=True)[:4]
    print(f"\n{tag} {dtype}: loss {lossv.item():.7f} vs fp64 {loss64:.7f} (rel {err_loss:.2e}), logits {err_logits:.2e}; "
          f"grad error vs fp64: engine median {med_eng:.2e}, reference {'bf16' if bf else 'fp32'} median {med_ref:.2e}; "
          f"worst engine/reference ratios {[(round(r, 2), nm) for r, nm in worst]}; "
          f"norm worst {max(norm_err.values()):.2e}")
    assert err_loss < (1e-3 if bf else 1e-5), err_loss
    assert err_logits < (3e-2 if bf else 1e-3), err_logits
    k, floor = (2.0, 1.0) if bf else (4.0, 2.0)
    bad = {n: (round(e_eng[n], 5), round(e_ref[n], 5)) for n in e_eng
           if e_eng[n] > max(k * e_ref[n], floor * med_ref)}
    assert not bad, bad
    assert med_eng <= (1.5 if bf else 2.0) * med_ref, (med_eng, med_ref)
    ntol = 5e-2 if bf else 1e-3
    bad = {n: v for n, v in norm_err.items() if v > (10 * ntol if n.endswith("up.bias") else ntol)}
    assert not bad, bad
    # mathematically-zero gradients: rounding noise, no larger than the reference's own (fp32 / bf16-autocast) noise
    # on the same biases (10x margin: it is noise, re-drawn by every summation order)
    big = {n: v for n, v in dead.items() if v[0] > 10 * v[1] + 1e-12}
    assert not big, big
    if not bf:
        hist = torch.bincount(logits.argmax(1).reshape(-1), minlength=C).cpu().numpy()
        assert np.abs(hist - g["argmax_hist"]).sum() <= 1e-4 * hist.sum()


# ---------------------------------------------------------------------------------------------------------------
# The same 96^3 B=2 steps against the fp64 oracle PINNED to the engine's own kink decisions
# ---------------------------------------------------------------------------------------------------------------
PINNED_TOL = {  # per parameter tensor, max|engine - oracle| / max|oracle| (tests.helpers.rel)
    "float32": 1e-4,   # fp32 storage, fp32 accumulation: rounding alone (measured r04a: worst 4.4e-5, c5 up.bias)
    # bf16 activation / weight / gradient storage, 2^-9 relative per rounding, ~40 roundings from the loss to the
    # first layer (measured r04a: worst 7.8e-2 c3 / 9.0e-2 c5, medians 2.5e-2 / 3.0e-2).  For scale: the
    # reference's OWN bf16-autocast step is 0.43-0.50 (median, L2) from fp64 on the same inputs
    # (tests/golden/fullgrad_*.npz) -- unpinned, so kink flips included
    "bfloat16": 0.15,
}
PINNED_MEDIAN = {"float32": 2e-5, "bfloat16": 5e-2}
PINNED_DEAD = {"float32": 1e-5, "bfloat16": 2e-2}    # of the largest gradient (measured 2.8e-7 / 6.5e-3)


def _oracle_fwd(kind, mods):
    from oracle import mmseg_oracle as O
    if kind == "unet":
        return lambda p, x, pins: O.unet3d_forward(p, x, 5, pins=pins)
    return lambda p, x, pins: O.dual_encoder_forward(p, x, "cross_attention", 5, pins=pins)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("tag,dtype,group", [("fullgrad_dual_c3", "float32", "1"), ("fullgrad_dual_c3", "bfloat16", "1"),
                                             ("fullgrad_unet_c2", "float32", "1"), ("fullgrad_dual_m3_c5", "float32", "1"),
                                             ("fullgrad_dual_m3_c5", "bfloat16", "1"),
                                             ("fullgrad_dual_c3", "bfloat16", "0"),
                                             ("fullgrad_dual_c3", "bfloat16", "noforce")])
def test_fullsize_step_pinned_to_fp64_oracle(dev, tag, dtype, group, monkeypatch):
    """The benched step at full size (96^3, B=2; trainer.py:250-254) against oracle/mmseg_oracle.py evaluated in
    fp64 ON THE GPU (torch ops) with the engine's own ReLU masks and MaxPool argmax codes (oracle.Pins, as
    tests/test_model_gpu.py does for the tiny configs).  At 96^3 a ReLU / MaxPool decision within rounding of its
    kink re-routes one voxel's gradient discretely, which is why the free comparison above needs bounds relative
    to the reference's own noise; with the decisions pinned the oracle and the engine differ by rounding alone,
    so EVERY parameter gradient is held to PINNED_TOL (fp32: 1e-4), including the ConvTranspose biases; the conv
    biases in front of an InstanceNorm (true gradient 0) to PINNED_DEAD of the largest gradient."""
    from tests.test_model_gpu import _engine_pins
    # "1" (default): the modality-grouped levels -- 12^3 / 6^3, and with MMSEG_GROUP_FORCE_R (default on) 24^3 / 48^3
    # on the runtime-brick kernels; "noforce": only 12^3 / 6^3; "0": every level per modality
    monkeypatch.setenv("MMSEG_GROUP_SMALL", "0" if group == "0" else "1")
    monkeypatch.setenv("MMSEG_GROUP_FORCE_R", "0" if group == "noforce" else "1")
    g = golden(tag)
    model, mods, loss = CASES[tag]
    S, B, seed, C = int(g["S"]), int(g["B"]), int(g["seed"]), 6
    cfg = _config(model, mods, loss, dtype)
    torch.manual_seed(seed)
    m = build_model(cfg)
    x, y, _ = full_inputs(S, B, len(mods), C, seed)
    x, y = x.to(dev), y.to(dev)
    tr = Trainer(cfg, m)
    m.train()
    lossv = tr._fused_loss(x, y)
    assert lossv is not None, "fused head + loss path not taken"
    if model == "dual_encoder":
        # bf16: the 12^3 and 6^3 levels grouped over the modalities (the runtime-brick kernels are bf16-only, so
        # the fp32 parity mode keeps per-modality launches there)
        prog = m.backbone.__dict__["_engine"].program
        if group == "0" or dtype != "bfloat16":
            assert prog.l0 == prog.L, prog.l0
        elif group == "noforce":
            assert prog.l0 == 3, prog.l0
        else:                           # 24^3 and (c3 / c5 features) 48^3 grouped as well
            assert prog.l0 <= 2, prog.l0
    pins = _engine_pins(m, model)
    pins.relu_masks = [r.to(dev) for r in pins.relu_masks]
    pins.pool_codes = [c.to(dev) for c in pins.pool_codes]
    lossv.backward()
    torch.cuda.synchronize()
    import time
    t0 = time.time()
    from oracle import mmseg_oracle as O
    params = {n: p.detach().double().requires_grad_(True) for n, p in m.backbone.named_parameters()}
    lossf = O.dice_ce_loss if loss == "dice_ce" else O.tversky_loss
    with torch.backends.cudnn.flags(enabled=False):
        ro = _oracle_fwd(model, mods)(params, x.double(), pins)
        rl = lossf(ro, y)
        rl.backward()
    torch.cuda.synchronize()
    t_orc = time.time() - t0
    assert pins.ri == len(pins.relu_masks) and pins.pi == len(pins.pool_codes)
    errs, dead, l2 = {}, {}, {}
    gmax = max(float(p.grad.abs().max()) for p in params.values())
    for n, p in m.backbone.named_parameters():
        if n.endswith(("conv1.bias", "conv2.bias")):
            dead[n] = float(p.grad.abs().max()) / gmax
        else:
            errs[n] = rel(p.grad, params[n].grad)
            l2[n] = float((p.grad.double() - params[n].grad).norm() / params[n].grad.norm())
    del ro, params
    med = float(np.median(list(errs.values())))
    worst = sorted(((v, n) for n, v in errs.items()), reverse=True)[:4]
    err_loss = abs(lossv.item() - rl.item()) / abs(rl.item())
    print(f"\n{tag} {dtype} group={group} pinned fp64 oracle ({t_orc:.0f} s on the GPU): loss rel {err_loss:.2e}; grad errors "
          f"median {med:.2e}, worst {[(float(f'{v:.2e}'), n) for v, n in worst]}; L2 median "
          f"{float(np.median(list(l2.values()))):.2e} max {max(l2.values()):.2e}; dead-bias max "
          f"{max(dead.values()):.2e} of the largest gradient")
    tol = PINNED_TOL[dtype]
    assert err_loss < (1e-6 if dtype == "float32" else 1e-3), err_loss
    assert max(errs.values()) < tol, worst
    assert med < PINNED_MEDIAN[dtype], med
    assert max(dead.values()) < PINNED_DEAD[dtype], dead


def test_group_force_runs_other_kernels(dev, monkeypatch):
    """Why group=1 and group=noforce above are two checks, not one: forced grouping (MMSEG_GROUP_FORCE_R, default)
    runs the 48^3 / 24^3 encoder levels as ONE launch over both modalities on the runtime-brick kernels
    (conv3_brickr / wgrad_brickr), while noforce runs them per modality on the (4, 8, 8)-brick family (brick2 /
    brick8 / brick3 / wgrad_dma), whose split-K and accumulation orders differ.  Same bf16 c3 step, both modes in
    one process on the same inputs and weights: the launched kernel families differ, and the gradients differ by
    fp32 accumulation order only (not bitwise; L2 ~1e-7) -- each mode is held to the pinned fp64 oracle by the
    parametrized test, whose printed error profiles therefore agree to the digits shown."""
    from mmseg_amd.engine.profiler import TIMER
    model, mods, loss = CASES["fullgrad_dual_c3"]
    x, y, _ = full_inputs(96, 2, 2, 6, 11)
    x, y = x.to(dev), y.to(dev)
    # noforce's per-modality 24^3 64-column convs are 108 (4, 8, 8) bricks: under MMSEG_BRICK2_MINUNITS (default 128)
    # they would take the runtime brick with chunk splits -- a third decomposition (measured 7.75e-5 from force,
    # both modes still deterministic run to run and pinned above).  Held at 0 so noforce is the brick2 family the
    # docstring names.
    monkeypatch.setenv("MMSEG_BRICK2_MINUNITS", "0")
    out = {}
    for mode in ("1", "noforce"):
        monkeypatch.setenv("MMSEG_GROUP_FORCE_R", "0" if mode == "noforce" else "1")
        cfg = _config(model, mods, loss, "bfloat16")
        torch.manual_seed(3)
        m = build_model(cfg)
        tr = Trainer(cfg, m)
        m.train()
        TIMER.start()
        try:
            lossv = tr._fused_loss(x, y)
            lossv.backward()
        finally:
            TIMER.stop()          # (a failure here must not leave the timer on for later tests: it disables graphs)
        fams = {}
        for fam, *_ in TIMER.records():
            fams[fam] = fams.get(fam, 0) + 1
        prog = m.backbone.__dict__["_engine"].program
        out[mode] = (prog.l0, fams, torch.cat([p.grad.reshape(-1).float() for p in m.parameters()]).clone(),
                     float(lossv))
        del m, tr
    (l0f, ff, gf, lf), (l0n, fn, gn, ln) = out["1"], out["noforce"]
    only_f = sorted(k for k in ff if ff[k] != fn.get(k, 0))
    only_n = sorted(k for k in fn if fn[k] != ff.get(k, 0))
    d = float((gf - gn).norm() / gn.norm())
    print(f"\nforced grouping: l0 {l0f} vs {l0n}; launch counts that differ: force {[(k, ff[k]) for k in only_f]} / "
          f"noforce {[(k, fn[k]) for k in only_n]}; loss {lf:.6f} vs {ln:.6f}; gradient L2 difference {d:.2e}")
    assert l0f <= 2 and l0n == 3
    assert any(k.startswith("conv3_brickr_kernel<BN64>") for k in only_f)
    assert any(k.startswith(("conv3_brick2_kernel", "conv3_brick8_kernel", "wgrad_dma_kernel")) for k in only_n)
    # measured (r05d): 9.1e-8 -- the two kernel families differ only in fp32 accumulation order, which almost never
    # moves a bf16-rounded activation, so the pinned test above prints the same digits for both modes
    assert 0.0 < d < 1e-5, d
    assert abs(lf - ln) / abs(ln) < 1e-5


# ---------------------------------------------------------------------------------------------------------------
# c5 in mixed bf16 / fp8 (hardware.fp8: true) at full size
# ---------------------------------------------------------------------------------------------------------------
def test_fullsize_c5_fp8_step(dev):
    """Config c5 (DualEncoder CT+PET+MRI, Tversky, 96^3, B=2) with the e4m3 forward convolutions (bench.py
    --fp8), against the reference's own step on the same inputs (tests/golden/fullgrad_dual_m3_c5.npz) and
    against the engine's bf16 step.  e4m3 keeps 3 mantissa bits, so the bound is stated against the
    reference's own mixed precision: per parameter tensor e(x) = ||x - ref_fp64|| / ||ref_fp64|| on the
    fixture's sampled positions.  On these random inputs the gradients are ill-conditioned: the reference's own
    bf16-autocast step sits at a median e of 0.46 and the engine's bf16 step at 0.44; the e4m3 forward (3 mantissa
    bits, 12 % normwise on the logits) measures 0.91 (r04d), so the bound is 2.5x the reference's median -- fp8
    roughly doubles the gradient noise of bf16 here, which is why it stays opt-in (and buys no time: DESIGN).
    Loss within 1e-2 of fp64, the sampled logits within 0.2 normwise of fp64 and of the bf16 engine."""
    tag = "fullgrad_dual_m3_c5"
    g = golden(tag)
    model, mods, loss = CASES[tag]
    S, B, seed, C = int(g["S"]), int(g["B"]), int(g["seed"]), 6
    x, y, idx = full_inputs(S, B, len(mods), C, seed)
    x, y = x.to(dev), y.to(dev)
    res = {}
    for fp8 in (False, True):
        cfg = _config(model, mods, loss, "bfloat16")
        cfg["hardware"]["fp8"] = fp8
        torch.manual_seed(seed)
        m = build_model(cfg)
        tr = Trainer(cfg, m)
        m.train()
        lossv = tr._fused_loss(x, y)
        if lossv is None:                 # the e4m3 forward keeps the unfused head + loss
            lossv = tr.criterion(m(x), y)
        lossv.backward()
        if fp8:
            prog = m.backbone.__dict__["_engine"].program
            assert all(prog.encs[k][0].c2._f8 is not None for k in range(3)) and prog.dec.blocks[-1].c2._f8 is not None
        with torch.no_grad():
            logits = m(x)
        torch.cuda.synchronize()
        names = [n for n, _ in m.backbone.named_parameters()]
        bb = dict(m.backbone.named_parameters())
        off = g["gs_off"]
        e = {}
        for i, n in enumerate(names):
            if n.endswith(("conv1.bias", "conv2.bias")):
                continue
            sl = slice(off[i], off[i + 1])
            gi = torch.from_numpy(g["gs_idx"][sl]).to(dev)
            e[n] = _l2(bb[n].grad.reshape(-1)[gi].double().cpu().numpy(), g["gs_val64"][sl])
        samp = logits.reshape(B, C, -1)[:, :, torch.from_numpy(idx).to(dev)].double().cpu()
        res[fp8] = (lossv.item(), samp, e)
        del m, tr
    loss64 = float(g["loss64"])
    ref_bf = {n: _l2(g["gs_valbf"][slice(g["gs_off"][i], g["gs_off"][i + 1])],
                     g["gs_val64"][slice(g["gs_off"][i], g["gs_off"][i + 1])])
              for i, n in enumerate(g["param_names"]) if n in res[True][2]}
    l64 = torch.from_numpy(g["sample_logits64"])
    nrel = lambda a, b: float((a - b).norm() / b.norm())  # noqa: E731
    med8, medb, medr = (float(np.median(list(res[True][2].values()))), float(np.median(list(res[False][2].values()))),
                        float(np.median(list(ref_bf.values()))))
    print(f"\nc5 96^3 fp8: loss {res[True][0]:.6f} (bf16 {res[False][0]:.6f}, fp64 {loss64:.6f}); sampled logits vs fp64 "
          f"{nrel(res[True][1], l64):.3f} (bf16 engine {nrel(res[False][1], l64):.4f}), fp8 vs bf16 engine "
          f"{nrel(res[True][1], res[False][1]):.3f}; gradient error vs fp64, median over tensors: fp8 {med8:.3f}, "
          f"bf16 engine {medb:.3f}, reference bf16 autocast {medr:.3f}")
    assert abs(res[True][0] - loss64) < 1e-2 * abs(loss64)
    assert nrel(res[True][1], l64) < 0.2 and nrel(res[True][1], res[False][1]) < 0.2
    assert med8 <= 2.5 * medr, (med8, medr)
