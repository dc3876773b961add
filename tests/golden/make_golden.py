"""Generate the golden fixtures under tests/golden/ by running the REFERENCE
(wittyseok/multimodal-organ-segmentation, mounted read-only at /root/reference)
on the CPU of the build container.

Run once, here (the reference never travels to the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Only data is written (inputs + expected outputs as .npz); no reference source
is copied.  The reference is imported in place; `nibabel` is absent in this
image, so a two-class stub is put in sys.modules before `src.utils` is touched
(only the trainer imports need it; no NIfTI I/O happens).
"""
from __future__ import annotations

import os
import sys
import tempfile
import types

import numpy as np
import torch

REF = os.environ.get("MMSEG_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))


def _import_reference():
    sys.dont_write_bytecode = True
    if "nibabel" not in sys.modules:
        nib = types.ModuleType("nibabel")
        nib.Nifti1Header = type("Nifti1Header", (), {})
        nib.Nifti1Image = type("Nifti1Image", (), {})
        sys.modules["nibabel"] = nib
    sys.path.insert(0, REF)
    import src.models.build as build  # noqa: E402
    import src.trainer.losses as losses  # noqa: E402
    import src.trainer.metrics as metrics  # noqa: E402
    import src.trainer.trainer as trainer  # noqa: E402
    import src.models.fusion.attention_fusion as attn  # noqa: E402
    return build, losses, metrics, trainer, attn


build, losses, metrics, trainer_mod, attn_mod = _import_reference()


def base_config(model: str, modalities, out_channels: int, features, fusion="cross_attention",
                loss="dice_ce", lr=1e-3):
    return {
        "experiment": {"name": "golden", "output_dir": tempfile.mkdtemp(prefix="mmseg_golden_"), "seed": 0},
        "data": {"modalities": list(modalities)},
        "model": {"name": model, "in_channels": len(modalities), "out_channels": out_channels,
                  "backbone": {"features": list(features), "norm": "instance"},
                  "fusion": {"type": fusion}, "head": {"dropout": 0.0}},
        "training": {"epochs": 1, "batch_size": 2, "accumulation_steps": 1,
                     "optimizer": {"name": "adamw", "lr": lr, "weight_decay": 1e-5, "betas": [0.9, 0.999]},
                     "scheduler": {"name": "none"},
                     "loss": {"name": loss, "dice_weight": 0.5, "ce_weight": 0.5, "class_weights": None}},
        "hardware": {"device": "cpu", "mixed_precision": False},
    }


def param_summary(named):
    names, sums, abss, samp = [], [], [], []
    for k, v in named:
        v = v.detach().double().flatten()
        names.append(k)
        sums.append(v.sum().item())
        abss.append(v.abs().sum().item())
        idx = torch.linspace(0, v.numel() - 1, 16).long()
        samp.append(v[idx].numpy())
    return np.array(names), np.array(sums), np.array(abss), np.stack(samp)


def model_case(tag, cfg, S, B, seed=0, steps=3, full_logits=False):
    """Forward + loss + grads at init, then a `steps`-batch reference Trainer epoch."""
    torch.manual_seed(seed)
    model = build.build_model(cfg)
    M = len(cfg["data"]["modalities"])
    C = cfg["model"]["out_channels"]
    g = torch.Generator().manual_seed(seed + 1)
    xs = torch.randn(steps + 1, B, M, S, S, S, generator=g)
    ys = torch.randint(0, C, (steps + 1, B, S, S, S), generator=g)
    init_names, init_sum, init_abs, init_samp = param_summary(model.backbone.named_parameters())

    crit = losses.get_loss(cfg)
    model.train()
    out = model(xs[0])
    loss = crit(out, ys[0])
    loss.backward()
    g_names, g_sum, g_abs, g_samp = param_summary((k, p.grad) for k, p in model.backbone.named_parameters())
    gnorm = np.array([p.grad.double().norm().item() for _, p in model.backbone.named_parameters()])
    model.zero_grad(set_to_none=True)

    # reference Trainer: per-batch body of _train_epoch (trainer.py:231-261) over `steps` batches
    tr = trainer_mod.Trainer(config=cfg, model=model)
    recorded = []
    orig = tr.criterion

    def rec(o, t):
        l = orig(o, t)
        recorded.append(l.item())
        return l

    tr.criterion = rec
    tr.train_loader = [{"image": xs[1 + i], "label": ys[1 + i]} for i in range(steps)]
    tr._train_epoch()
    with torch.no_grad():
        model.eval()
        out_after = model(xs[0])
    # inputs are NOT stored: tests regenerate them from the same seeded CPU generator
    # (torch.Generator().manual_seed(seed + 1); randn then randint, shapes as above)
    flat = out.detach().reshape(-1)
    sidx = torch.randperm(flat.numel(), generator=torch.Generator().manual_seed(99))[:4096]
    extra = {"logits": out.detach().numpy()} if full_logits else {}
    np.savez_compressed(
        os.path.join(OUT, f"{tag}.npz"), S=np.int64(S), B=np.int64(B), steps=np.int64(steps),
        logits_sum=np.float64(out.detach().double().sum()), logits_abs=np.float64(out.detach().double().abs().sum()),
        sample_idx=sidx.numpy(), sample_logits=flat[sidx].numpy(), loss=np.float64(loss.item()), **extra,
        init_names=init_names, init_sum=init_sum, init_abs=init_abs, init_samp=init_samp,
        grad_sum=g_sum, grad_abs=g_abs, grad_samp=g_samp, grad_norm=gnorm,
        traj_losses=np.array(recorded), after_sample=out_after.reshape(-1)[sidx].numpy(),
        after_sum=np.float64(out_after.double().sum()),
        features=np.array(cfg["model"]["backbone"]["features"]), seed=np.int64(seed),
    )
    print(tag, "loss", loss.item(), "traj", recorded)


def loss_case():
    g = torch.Generator().manual_seed(7)
    out = {}
    for C in (3, 6, 7):
        logits = (torch.randn(2, C, 8, 9, 10, generator=g) * 3).requires_grad_(True)
        labels = torch.randint(0, C, (2, 8, 9, 10), generator=g)
        out[f"logits_C{C}"] = logits.detach().numpy()
        out[f"labels_C{C}"] = labels.numpy()
        cw = torch.rand(C, generator=g) + 0.5
        out[f"cw_C{C}"] = cw.numpy()
        mods = {
            "dicece": losses.DiceCELoss(),
            "dicece_w": losses.DiceCELoss(dice_weight=0.3, ce_weight=0.7, class_weights=cw),
            "dice": losses.DiceLoss(),
            "dice_nobg": losses.DiceLoss(include_background=False),
            "ce": torch.nn.CrossEntropyLoss(),
            "tversky": losses.TverskyLoss(),
            "tversky_37": losses.TverskyLoss(alpha=0.3, beta=0.7),
            "focal": losses.FocalLoss(),
            "focal_w": losses.FocalLoss(alpha=cw),
        }
        for name, mod in mods.items():
            if logits.grad is not None:
                logits.grad = None
            l = mod(logits, labels)
            l.backward()
            out[f"{name}_C{C}"] = np.float64(l.item())
            out[f"{name}_C{C}_grad"] = logits.grad.numpy().copy()
    np.savez_compressed(os.path.join(OUT, "losses.npz"), **out)
    print("losses done")


def metric_case():
    rng = np.random.default_rng(11)
    out = {}
    for C in (3, 6):
        dm = metrics.DiceMetric(num_classes=C)
        preds, tgts = [], []
        for _ in range(3):
            p = rng.integers(0, C, size=(2, 12, 12, 12))
            t = rng.integers(0, C, size=(2, 12, 12, 12))
            if C == 6:
                p[p == 5] = 4  # class 5 absent from predictions
                t[t == 5] = 4  # ... and from targets: absent class -> dice 1.0
            preds.append(p)
            tgts.append(t)
            dm.update(torch.from_numpy(p), torch.from_numpy(t))
        res = dm.compute()
        out[f"pred_C{C}"] = np.stack(preds)
        out[f"tgt_C{C}"] = np.stack(tgts)
        out[f"inter_C{C}"] = dm.intersection.numpy()
        out[f"union_C{C}"] = dm.union.numpy()
        out[f"dice_C{C}"] = np.float64(res["dice"])
        out[f"dpc_C{C}"] = np.array(res["dice_per_class"])
    np.savez_compressed(os.path.join(OUT, "dice_metric.npz"), **out)
    print("metric done")


def cross_attention_case():
    torch.manual_seed(3)
    mod = attn_mod.CrossAttentionFusion(32, num_heads=4)
    g = torch.Generator().manual_seed(4)
    q = torch.randn(2, 32, 6, 6, 6, generator=g).requires_grad_(True)
    kv = torch.randn(2, 32, 6, 6, 6, generator=g).requires_grad_(True)
    o = mod(q, kv)
    w = torch.randn(o.shape, generator=g)
    (o * w).sum().backward()
    sd = {k: v.detach().numpy() for k, v in mod.state_dict().items()}
    np.savez_compressed(os.path.join(OUT, "cross_attention.npz"), q=q.detach().numpy(), kv=kv.detach().numpy(),
                        out=o.detach().numpy(), cot=w.numpy(), dq=q.grad.numpy(), dkv=kv.grad.numpy(),
                        **{"p_" + k: v for k, v in sd.items()},
                        **{"g_" + k: p.grad.numpy() for k, p in mod.named_parameters()})
    print("cross attention done")


def bidirectional_case():
    """BidirectionalCrossAttention (attention_fusion.py:167-216): two CrossAttentionFusion + 2C->C 1x1 conv,
    InstanceNorm3d, ReLU; forward, input and parameter gradients at 6^3, C=32, 4 heads."""
    torch.manual_seed(5)
    mod = attn_mod.BidirectionalCrossAttention(32, num_heads=4)
    g = torch.Generator().manual_seed(6)
    f1 = torch.randn(2, 32, 6, 6, 6, generator=g).requires_grad_(True)
    f2 = torch.randn(2, 32, 6, 6, 6, generator=g).requires_grad_(True)
    o = mod(f1, f2)
    w = torch.randn(o.shape, generator=g)
    (o * w).sum().backward()
    np.savez_compressed(os.path.join(OUT, "bidirectional_attention.npz"), f1=f1.detach().numpy(),
                        f2=f2.detach().numpy(), out=o.detach().numpy(), cot=w.numpy(), d1=f1.grad.numpy(),
                        d2=f2.grad.numpy(), **{"p_" + k: v.detach().numpy() for k, v in mod.state_dict().items()},
                        **{"g_" + k: p.grad.numpy() for k, p in mod.named_parameters()})
    print("bidirectional attention done")


def transforms_case():
    """ModalitySpecificNormalize (transforms.py:362-404) + Resize (transforms.py:215-250, scipy zoom order 1 /
    labels order 0) on a small raw CT (HU) / PET (SUV) / MRI sample, non-cubic and resized up and down."""
    import src.data.transforms as T
    rng = np.random.Generator(np.random.PCG64(77))
    shape = (20, 24, 28)
    ct = rng.uniform(-1200, 1500, shape).astype(np.float32)
    pet = np.abs(rng.normal(2.0, 3.0, shape)).astype(np.float32)
    mri = rng.normal(300.0, 80.0, shape).astype(np.float32)
    image = np.stack([ct, pet, mri])
    label = rng.integers(0, 5, size=shape).astype(np.int64)
    cfg = {"data": {"modalities": ["CT", "PET", "MRI"],
                    "preprocessing": {"ct": {"window_center": -100, "window_width": 700},
                                      "pet": {"normalize": True}, "mri": {"normalize": True}}}}
    norm = T.ModalitySpecificNormalize(cfg)({"image": image.copy()})["image"]
    out = {"image_in": image, "label_in": label, "normalized": norm}
    for name, size in (("up", (32, 30, 36)), ("down", (12, 16, 9))):
        r = T.Resize(size, order=1)({"image": norm.copy(), "label": label.copy()})
        out[f"resized_{name}"] = r["image"]
        out[f"label_{name}"] = r["label"]
        out[f"size_{name}"] = np.array(size, dtype=np.int64)
    np.savez_compressed(os.path.join(OUT, "transforms.npz"), **out)
    print("transforms done", norm.dtype, out["resized_up"].dtype, out["label_up"].dtype)


def full_case(tag, cfg, S, B, seed):
    """Full-size configs: forward summary only (logits stats + seeded voxel samples)."""
    torch.manual_seed(seed)
    model = build.build_model(cfg)
    M = len(cfg["data"]["modalities"])
    C = cfg["model"]["out_channels"]
    rng = np.random.Generator(np.random.PCG64(seed + 100))
    x = torch.from_numpy(rng.standard_normal((B, M, S, S, S), dtype=np.float32))
    y = torch.from_numpy(rng.integers(0, C, size=(B, S, S, S)).astype(np.int64))
    with torch.no_grad():
        out = model(x)
        loss = losses.get_loss(cfg)(out, y)
    flat = out.reshape(B, C, -1)
    idx = rng.integers(0, S ** 3, size=1024)
    names, psum, pabs, _ = param_summary(model.backbone.named_parameters())
    np.savez_compressed(os.path.join(OUT, f"{tag}.npz"), S=np.int64(S), B=np.int64(B), seed=np.int64(seed),
                        logits_sum=np.float64(out.double().sum()), logits_abs=np.float64(out.double().abs().sum()),
                        logits_absmax=np.float64(out.abs().max()), sample_idx=idx,
                        sample_logits=flat[:, :, idx].numpy(), loss=np.float64(loss.item()),
                        argmax_hist=np.bincount(out.argmax(1).flatten().numpy(), minlength=C),
                        param_names=names, param_sum=psum, param_abs=pabs)
    print(tag, "loss", loss.item())


def grad_sample_index(numel: int, k: int, seed: int) -> np.ndarray:
    """Seeded positions at which a gradient tensor is sampled (all positions when it has <= k elements).
    Tests regenerate the same positions from (numel, k, seed)."""
    if numel <= k:
        return np.arange(numel, dtype=np.int64)
    rng = np.random.Generator(np.random.PCG64(seed))
    return np.sort(rng.choice(numel, size=k, replace=False)).astype(np.int64)


def full_inputs(S, B, M, C, seed):
    """Data-only full-size inputs (shared by full_case / full_grad_case and the tests)."""
    rng = np.random.Generator(np.random.PCG64(seed + 100))
    x = torch.from_numpy(rng.standard_normal((B, M, S, S, S), dtype=np.float32))
    y = torch.from_numpy(rng.integers(0, C, size=(B, S, S, S)).astype(np.int64))
    idx = rng.integers(0, S ** 3, size=1024)
    return x, y, idx


def full_grad_case(tag, cfg, S, B, seed, k=4096):
    """Full-size TRAINING step of the reference (trainer.py:250-254 with accumulation 1): train-mode forward,
    the configured loss, backward.  Stored: loss, 1024 seeded voxels of every logit channel, the argmax
    histogram, and per parameter gradient its L2 norm, sum and the values at k seeded positions (all of them
    for tensors with <= k elements).  Initial weights are reproduced by torch.manual_seed(seed) + build_model."""
    M = len(cfg["data"]["modalities"])
    C = cfg["model"]["out_channels"]
    x, y, idx = full_inputs(S, B, M, C, seed)
    crit = losses.get_loss(cfg)

    def run(mode):
        """mode f32: the reference as it runs on CPU; f64: the same step in double (its rounding-free answer);
        bf16: under torch.autocast("cpu", bfloat16), the CPU analogue of the reference's own mixed-precision
        step (trainer.py:237-243 autocasts in fp16 on a GPU).  The f64 / bf16 runs measure how far rounding
        alone moves these gradients: at 96^3 a few hundred ReLU / MaxPool decisions per layer sit within rounding
        of their kink (fp32), tens of thousands at bf16, and every weight gradient is a heavily cancelling sum
        over 1.8 M voxels."""
        torch.manual_seed(seed)
        model = build.build_model(cfg)
        if mode == "f64":
            model = model.double()
        model.train()
        xin = x.double() if mode == "f64" else x
        if mode == "bf16":
            with torch.autocast("cpu", dtype=torch.bfloat16):
                out = model(xin)
            loss = crit(out.float(), y)
        else:
            out = model(xin)
            loss = crit(out, y)
        loss.backward()
        res = {"loss": loss.item(), "out": out.detach().float(), "names": [], "norms": [], "sums": [], "sidx": [],
               "sval": []}
        for i, (n, p) in enumerate(model.backbone.named_parameters()):
            g = p.grad.detach().double().reshape(-1)
            res["names"].append(n)
            res["norms"].append(g.norm().item())
            res["sums"].append(g.sum().item())
            gi = grad_sample_index(g.numel(), k, seed * 1000 + i)
            res["sidx"].append(gi)
            res["sval"].append(g[torch.from_numpy(gi)].numpy())
        return res

    r32, r64, rbf = run("f32"), run("f64"), run("bf16")
    out = r32["out"]
    soff = np.cumsum([0] + [len(v) for v in r32["sidx"]])
    flat = out.reshape(B, C, -1)
    np.savez_compressed(os.path.join(OUT, f"{tag}.npz"), S=np.int64(S), B=np.int64(B), seed=np.int64(seed),
                        k=np.int64(k), loss=np.float64(r32["loss"]), loss64=np.float64(r64["loss"]),
                        lossbf=np.float64(rbf["loss"]), sample_idx=idx,
                        sample_logits=flat[:, :, idx].numpy(),
                        sample_logits64=r64["out"].reshape(B, C, -1)[:, :, idx].numpy(),
                        logits_sum=np.float64(out.double().sum()),
                        argmax_hist=np.bincount(out.argmax(1).flatten().numpy(), minlength=C),
                        param_names=np.array(r32["names"]), grad_norm=np.array(r32["norms"]),
                        grad_norm64=np.array(r64["norms"]), grad_sum=np.array(r32["sums"]),
                        gs_idx=np.concatenate(r32["sidx"]), gs_val=np.concatenate(r32["sval"]),
                        gs_val64=np.concatenate(r64["sval"]), gs_valbf=np.concatenate(rbf["sval"]),
                        gs_off=soff)
    e32 = [np.linalg.norm(a - b) / np.linalg.norm(b) for a, b in zip(r32["sval"], r64["sval"])]
    ebf = [np.linalg.norm(a - b) / np.linalg.norm(b) for a, b in zip(rbf["sval"], r64["sval"])]
    print(tag, "loss", r32["loss"], r64["loss"], rbf["loss"], "params", len(r32["names"]),
          f"grad err vs f64: f32 median {np.median(e32):.2e} max {max(e32):.2e}; "
          f"bf16 median {np.median(ebf):.2e} max {max(ebf):.2e}")


def _phantom_batch(seed, S, C, mods, class_seed=None):
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(OUT)), "multimodal-organ-segmentation_amd",
                                    "data"))
    from synthetic import phantom    # the repo's seeded numpy phantom (plain data generation)
    p = phantom(int(seed), S, C, mods, class_seed=class_seed)
    return {"image": torch.from_numpy(np.stack([p[m] for m in mods]))[None],
            "label": torch.from_numpy(p["label"])[None]}


def dice_heldout_case(K=16, V=2, S=64, lr=1e-4):
    """north_star "Dice on a held-out synthetic set": config c1 (UNet3D, CT+PET, 3 classes, 64^3, batch 1,
    DiceCE, AdamW lr 1e-4 = the c1 / default.yaml rate).  The reference Trainer runs one epoch over K phantom
    batches (train seeds 1234..1234+K-1, trainer.py:222-263), then _validate (trainer.py:265-296: argmax +
    DiceMetric, metrics.py:42-88) on V held-out phantoms (seeds 4321..).  The same run in fp64 is stored as the
    reference's own rounding spread: a free-running K-step trajectory amplifies fp32 rounding (AdamW's first
    steps move weights by ~lr * sign(g) wherever g is tiny), so two correct fp32 implementations differ by
    about |ref32 - ref64| in held-out Dice."""
    mods = ["CT", "PET"]
    out = {"K": np.int64(K), "V": np.int64(V), "S": np.int64(S), "lr": np.float64(lr),
           "train_seeds": np.arange(1234, 1234 + K), "val_seeds": np.arange(4321, 4321 + V)}
    for dt, tag in ((torch.float32, "f32"), (torch.float64, "f64")):
        cfg = base_config("unet", mods, 3, [32, 64, 128, 256, 512], lr=lr)
        torch.manual_seed(42)
        model = build.build_model(cfg).to(dt)
        tr = trainer_mod.Trainer(config=cfg, model=model)
        cast = lambda b: {"image": b["image"].to(dt), "label": b["label"]}  # noqa: E731
        tr.train_loader = [cast(_phantom_batch(s, S, 3, mods)) for s in out["train_seeds"]]
        tr.val_loader = [cast(_phantom_batch(s, S, 3, mods)) for s in out["val_seeds"]]
        recorded = []
        orig = tr.criterion

        def rec(o, t, orig=orig, recorded=recorded):
            lv = orig(o, t)
            recorded.append(lv.item())
            return lv
        tr.criterion = rec
        tr._train_epoch()
        tr.criterion = orig
        # _validate's DiceMetric is local: recompute its counts with the same calls to store I / U
        dm = metrics.DiceMetric(num_classes=3)
        model.eval()
        with torch.no_grad():
            for b in tr.val_loader:
                dm.update(torch.argmax(model(b["image"]), dim=1), b["label"])
        vloss, met = tr._validate()
        out[f"{tag}_train_losses"] = np.array(recorded)
        out[f"{tag}_val_loss"] = np.float64(vloss)
        out[f"{tag}_dice"] = np.float64(met["dice"])
        out[f"{tag}_dice_per_class"] = np.array(met["dice_per_class"])
        out[f"{tag}_inter"] = dm.intersection.numpy()
        out[f"{tag}_union"] = dm.union.numpy()
        assert abs(dm.compute()["dice"] - met["dice"]) == 0.0
        print("dice_heldout", tag, met, "val loss", vloss)
    np.savez_compressed(os.path.join(OUT, "dice_heldout_c1.npz"), **out)


def dice_heldout_trained_case(K=160, V=16, S=64, lr=2e-3, class_seed=77, feats=(8, 16, 32, 64, 128)):
    """Held-out Dice on the REFERENCE's trained weights (north_star "Dice on a held-out synthetic set matching
    reference +-1e-4").  UNet3D CT+PET, 3 classes, 64^3, batch 1, DiceCE, AdamW: the reference Trainer runs one
    epoch over K organ-consistent phantoms (class_seed: the organs' intensities are the same in every phantom,
    so the model learns which organ is which; train seeds 1234.., trainer.py:222-263), then _validate
    (trainer.py:265-296, DiceMetric metrics.py:42-88) on V held-out phantoms (seeds 4321..).  Stored: the
    trained weights (fp32, plain arrays -- the network is the c1 UNet3D at features 8..128 so they stay a
    small fixture), the reference's held-out Dice / per-class Dice / I / U / loss on them, its argmax masks
    (uint8) for flip counting, its training losses, and the same run in fp64 (the reference's own spread for
    the free-running comparison)."""
    mods = ["CT", "PET"]
    out = {"K": np.int64(K), "V": np.int64(V), "S": np.int64(S), "lr": np.float64(lr),
           "class_seed": np.int64(class_seed), "features": np.array(feats),
           "train_seeds": np.arange(1234, 1234 + K), "val_seeds": np.arange(4321, 4321 + V)}
    for dt, tag in ((torch.float32, "f32"), (torch.float64, "f64")):
        cfg = base_config("unet", mods, 3, list(feats), lr=lr)
        torch.manual_seed(42)
        model = build.build_model(cfg).to(dt)
        tr = trainer_mod.Trainer(config=cfg, model=model)
        cast = lambda b: {"image": b["image"].to(dt), "label": b["label"]}  # noqa: E731
        tr.train_loader = [cast(_phantom_batch(s, S, 3, mods, class_seed)) for s in out["train_seeds"]]
        tr.val_loader = [cast(_phantom_batch(s, S, 3, mods, class_seed)) for s in out["val_seeds"]]
        recorded = []
        orig = tr.criterion

        def rec(o, t, orig=orig, recorded=recorded):
            lv = orig(o, t)
            recorded.append(lv.item())
            return lv
        tr.criterion = rec
        tr._train_epoch()
        tr.criterion = orig
        dm = metrics.DiceMetric(num_classes=3)
        masks = []
        model.eval()
        with torch.no_grad():
            for b in tr.val_loader:
                pred = torch.argmax(model(b["image"]), dim=1)
                masks.append(pred[0].to(torch.uint8).numpy())
                dm.update(pred, b["label"])
        vloss, met = tr._validate()
        assert abs(dm.compute()["dice"] - met["dice"]) == 0.0
        out[f"{tag}_train_losses"] = np.array(recorded)
        out[f"{tag}_val_loss"] = np.float64(vloss)
        out[f"{tag}_dice"] = np.float64(met["dice"])
        out[f"{tag}_dice_per_class"] = np.array(met["dice_per_class"])
        out[f"{tag}_inter"] = dm.intersection.numpy()
        out[f"{tag}_union"] = dm.union.numpy()
        if tag == "f32":
            out["masks"] = np.stack(masks)
            names = [n for n, _ in model.named_parameters()]
            out["param_names"] = np.array(names)
            for i, (n, p) in enumerate(model.named_parameters()):
                out[f"w{i}"] = p.detach().numpy().astype(np.float32)
        print("dice_heldout_trained", tag, met, "val loss", vloss)
    np.savez_compressed(os.path.join(OUT, "dice_heldout_trained.npz"), **out)


def dice_heldout_envelope_case(threads=(1, 2, 4, 6)):
    """The reference's own reproducibility envelope for the two free-running held-out Dice checks
    (test_dice_heldout_gpu.py): the SAME reference runs as dice_heldout_case / dice_heldout_trained_case (stored
    there at 8 threads, fp32 and fp64), repeated in fp32 at other intra-op thread counts.  Each thread count
    changes the CPU kernels' summation order (blocked reductions in mkldnn convolutions and the loss), i.e. is
    another legitimate fp32 ordering of the same algorithm; the spread of held-out Dice over these orderings
    and fp64 is what a correct fp32 implementation with yet another summation order (the HIP engine) can
    differ by.  Stored per case: the thread counts and the Dice / train-loss trajectories of each run."""
    mods = ["CT", "PET"]
    cases = {"c1": dict(K=16, V=2, S=64, lr=1e-4, feats=[32, 64, 128, 256, 512], class_seed=None),
             "trained": dict(K=160, V=16, S=64, lr=2e-3, feats=[8, 16, 32, 64, 128], class_seed=77)}
    out = {"threads": np.array(threads)}
    for cname, c in cases.items():
        train = [_phantom_batch(s, c["S"], 3, mods, c["class_seed"]) for s in range(1234, 1234 + c["K"])]
        val = [_phantom_batch(s, c["S"], 3, mods, c["class_seed"]) for s in range(4321, 4321 + c["V"])]
        dices, losses = [], []
        for t in threads:
            torch.set_num_threads(int(t))
            cfg = base_config("unet", mods, 3, c["feats"], lr=c["lr"])
            torch.manual_seed(42)
            model = build.build_model(cfg)
            tr = trainer_mod.Trainer(config=cfg, model=model)
            tr.train_loader, tr.val_loader = train, val
            recorded = []
            orig = tr.criterion

            def rec(o, tt, orig=orig, recorded=recorded):
                lv = orig(o, tt)
                recorded.append(lv.item())
                return lv
            tr.criterion = rec
            tr._train_epoch()
            tr.criterion = orig
            vloss, met = tr._validate()
            dices.append(met["dice"])
            losses.append(recorded)
            print("dice_heldout_envelope", cname, "threads", t, met["dice"], "val loss", vloss, flush=True)
        out[f"{cname}_f32_dice"] = np.array(dices, dtype=np.float64)
        out[f"{cname}_f32_train_losses"] = np.array(losses, dtype=np.float64)
    torch.set_num_threads(8)
    np.savez_compressed(os.path.join(OUT, "dice_heldout_envelope.npz"), **out)


def checkpoint_case():
    """A checkpoint written by the reference (save_checkpoint, build.py:153-180: epoch, model_state_dict,
    optimizer_state_dict (torch AdamW), best_metric, history) after 2 Trainer steps of a small UNet3D
    (features [8, 16, 32], 32^3, B=2, 3 classes, lr 1e-3), and what the reference does next: a fresh model +
    Trainer(resume_from=...) (trainer.py:150-164) trains one more batch; its loss and the resulting parameters
    are stored.  The .pth holds only tensors / numbers / dicts / lists, so torch.load(weights_only=True)
    reads it.  Also stored: the reference's c1 UNet3D and c3 DualEncoder state-dict key lists + shapes (the
    checkpoint format an engine-written checkpoint must keep)."""
    feats = [8, 16, 32]
    cfg = base_config("unet", ["CT", "PET"], 3, feats, lr=1e-3)
    g = torch.Generator().manual_seed(31)
    xs = torch.randn(3, 2, 2, 32, 32, 32, generator=g)
    ys = torch.randint(0, 3, (3, 2, 32, 32, 32), generator=g)
    torch.manual_seed(0)
    model = build.build_model(cfg)
    tr = trainer_mod.Trainer(config=cfg, model=model)
    tr.train_loader = [{"image": xs[i], "label": ys[i]} for i in range(2)]
    tr._train_epoch()
    path = os.path.join(OUT, "ref_ckpt_unet_small.pth")
    build.save_checkpoint(model, tr.optimizer, epoch=3, checkpoint_path=path, best_metric=0.25,
                          history={"train_loss": [1.0], "val_loss": [1.1], "val_dice": [0.25]})
    torch.load(path, map_location="cpu", weights_only=True)     # the safe loader must accept it
    torch.manual_seed(123)                                      # a different init: everything comes from the file
    model2 = build.build_model(cfg)
    tr2 = trainer_mod.Trainer(config=cfg, model=model2, resume_from=path)
    recorded = []
    orig = tr2.criterion
    tr2.criterion = lambda o, t: recorded.append(orig(o, t)) or recorded[-1]
    tr2.train_loader = [{"image": xs[2], "label": ys[2]}]
    tr2._train_epoch()
    names = [n for n, _ in model2.named_parameters()]
    after = torch.cat([p.detach().reshape(-1) for p in model2.parameters()]).double()
    keys = {}
    for kind, mcfg in (("c1_unet", base_config("unet", ["CT", "PET"], 3, [32, 64, 128, 256, 512])),
                       ("c3_dual", base_config("dual_encoder", ["CT", "PET"], 6, [32, 64, 128, 256, 512]))):
        sd = build.build_model(mcfg).state_dict()
        keys[f"{kind}_keys"] = np.array(list(sd))
        keys[f"{kind}_shapes"] = np.array([",".join(map(str, v.shape)) for v in sd.values()])
    np.savez_compressed(os.path.join(OUT, "ref_ckpt_unet_small.npz"), next_loss=np.float64(recorded[0].item()),
                        resume_epoch=np.int64(tr2.current_epoch), after=after.numpy(), names=np.array(names),
                        **keys)
    print("checkpoint: next loss", recorded[0].item(), "resumed epoch", tr2.current_epoch)


def full_grad_cases():
    F = [32, 64, 128, 256, 512]
    full_grad_case("fullgrad_unet_c2", base_config("unet", ["CT", "PET"], 6, F), S=96, B=2, seed=1234)
    full_grad_case("fullgrad_dual_c3", base_config("dual_encoder", ["CT", "PET"], 6, F), S=96, B=2, seed=1234)
    full_grad_case("fullgrad_dual_m3_c5", base_config("dual_encoder", ["CT", "PET", "MRI"], 6, F, loss="tversky"),
                   S=96, B=2, seed=1234)


if __name__ == "__main__":
    torch.set_num_threads(8)
    if len(sys.argv) > 1:          # regenerate only the named cases, e.g. `make_golden.py bidirectional_case`
        for name in sys.argv[1:]:
            if name == "full_grad_cases":
                full_grad_cases()
            else:
                globals()[name]()
        sys.exit(0)
    feats = [8, 16, 32, 64, 128]
    model_case("unet_tiny", base_config("unet", ["CT", "PET"], 3, feats), S=32, B=2, full_logits=True)
    for fz in ("cross_attention", "concat", "add", "attention"):
        model_case(f"dual_tiny_{fz}", base_config("dual_encoder", ["CT", "PET"], 3, feats, fusion=fz), S=32, B=2)
    model_case("dual_tiny_m3_tversky", base_config("dual_encoder", ["CT", "PET", "MRI"], 6, feats,
                                                   fusion="cross_attention", loss="tversky"), S=32, B=2)
    loss_case()
    metric_case()
    cross_attention_case()
    transforms_case()
    full_case("full_unet_c2", base_config("unet", ["CT", "PET"], 6, [32, 64, 128, 256, 512]), S=96, B=2, seed=1234)
    full_case("full_dual_c3", base_config("dual_encoder", ["CT", "PET"], 6, [32, 64, 128, 256, 512]),
              S=96, B=2, seed=1234)
    full_grad_cases()
    dice_heldout_case()
    checkpoint_case()
