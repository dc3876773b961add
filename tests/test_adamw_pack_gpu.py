"""The fused AdamW + weight pack (mmseg_adamw_pack / _dev, conv_gemm.hip adamw_pack_kernel) against the two
launches it replaces: mmseg_adamw over the arena, then the engine's batched packs (layers.Packer.run) from the
updated fp32 weights.  Parameters, moments and every operand image must be BITWISE equal -- on UNet3D /
DualEncoder (3^3 conv tiles, transposed convs) and SwinUNETR (token linears, patch embedding, transposed convs,
channel-padded images), bf16 and fp32 images.  Then the trainer-level contract: the eager step with the fused
launch (the next forward skips its pack) equals the step that packs every forward, and weights changed through
torch (load_state_dict) are re-packed before the next forward reads them."""
import pytest
import torch

import mmseg_amd  # noqa: F401
from mmseg_amd._lib import lib, ptr, stream_handle
from mmseg_amd.models.build import build_model
from mmseg_amd.trainer.trainer import Trainer

pytestmark = pytest.mark.gpu


def _cfg(model, dtype, feats=(8, 16, 32, 64, 128)):
    m = {"name": model, "in_channels": 2, "out_channels": 3,
         "backbone": {"features": list(feats), "norm": "instance"},
         "fusion": {"type": "cross_attention"}, "head": {"dropout": 0.0}}
    if model == "swin_unetr":
        m = {"name": model, "in_channels": 2, "out_channels": 3,
             "backbone": {"img_size": [64, 64, 64], "feature_size": 24}}
    return {
        "experiment": {"name": "adamw_pack", "output_dir": "/tmp/mmseg_adamw_pack", "seed": 0},
        "data": {"modalities": ["CT", "PET"]},
        "model": m,
        "training": {"epochs": 1, "batch_size": 1, "accumulation_steps": 1,
                     "optimizer": {"name": "adamw", "lr": 1e-3, "weight_decay": 1e-5, "betas": [0.9, 0.999]},
                     "scheduler": {"name": "none"},
                     "loss": {"name": "dice_ce", "dice_weight": 0.5, "ce_weight": 0.5, "class_weights": None},
                     "checkpoint": {"save_last": False, "save_best": False}},
        "hardware": {"device": "cuda", "mixed_precision": dtype == "bfloat16", "engine_dtype": dtype,
                     "step_graph": False},
    }


def _size(model):
    return 64 if model == "swin_unetr" else 32


def _batch(dev, model, seed=3):
    S = _size(model)
    g = torch.Generator().manual_seed(seed)
    return {"image": torch.randn(1, 2, S, S, S, generator=g).to(dev),
            "label": torch.randint(0, 3, (1, S, S, S), generator=g).to(dev)}


def _engine(tr):
    bb = getattr(tr.model, "backbone", tr.model)
    return bb.__dict__["_engine"]


def _images(prog, ptrs):
    """The image tensors behind the Packer's destination pointers (walks the engine's layer objects)."""
    found, seen, stack = {}, set(), [prog]
    while stack:
        o = stack.pop()
        if id(o) in seen:
            continue
        seen.add(id(o))
        if isinstance(o, torch.Tensor):
            if o.is_cuda and o.data_ptr() in ptrs:
                found.setdefault(o.data_ptr(), o)
            continue
        if isinstance(o, (list, tuple)):
            stack.extend(o)
        elif isinstance(o, dict):
            stack.extend(o.values())
        elif hasattr(o, "__dict__") and not isinstance(o, (torch.nn.Module, type)):
            stack.extend(vars(o).values())
    assert set(found) == set(ptrs), f"{len(set(ptrs) - set(found))} image buffers not found"
    return found


@pytest.mark.parametrize("model,dtype", [("unet", "bfloat16"), ("unet", "float32"), ("dual_encoder", "bfloat16"),
                                         ("swin_unetr", "bfloat16"), ("swin_unetr", "float32")])
def test_adamw_pack_bitwise_equals_adamw_then_pack(dev, model, dtype):
    cfg = _cfg(model, dtype)
    torch.manual_seed(0)
    tr = Trainer(cfg, build_model(cfg))
    tr.train_step(_batch(dev, model), 0)            # builds the engine, the images and the moments
    eng = _engine(tr)
    flat, prog = eng.flat, eng.program
    pk = prog.packer()
    tab = pk.adam(flat)
    assert tab is not None, "every weight of the model fits the fused kinds"
    rows = tab[0].view(-1, lib().mmseg_adamw_pack_desc_bytes())[:, 24:28].contiguous()
    kinds = {int(k) for k in rows.view(torch.int32).view(-1).cpu()}
    assert 0 in kinds and 2 in kinds and (1 in kinds or model != "swin_unetr")
    imgs = _images(prog, {d[1] for d in pk.descs})
    n = flat.numel
    m, v = tr.optimizer._flat[0]
    g = torch.Generator(device=dev).manual_seed(7)
    flat.grad_flat.copy_(torch.randn(n, device=dev, generator=g) * 0.05)
    m.copy_(torch.randn(n, device=dev, generator=g) * 1e-2)
    v.copy_(torch.rand(n, device=dev, generator=g) * 1e-3)
    p0, m0, v0 = flat.flat.clone(), m.clone(), v.clone()
    img0 = {k: t.clone() for k, t in imgs.items()}
    hyper = (0.05, 0.9, 0.999, 1e-8, 1e-2, 3)       # lr large enough that every bf16 image entry moves
    L, s = lib(), stream_handle()

    L.mmseg_adamw(ptr(flat.flat), ptr(flat.grad_flat), ptr(m), ptr(v), n, *hyper, None, s)
    pk.run()
    torch.cuda.synchronize()
    ref = (flat.flat.clone(), m.clone(), v.clone(), {k: t.clone() for k, t in imgs.items()})

    flat.flat.copy_(p0), m.copy_(m0), v.copy_(v0)
    for k, t in imgs.items():
        t.copy_(img0[k])
    L.mmseg_adamw_pack(ptr(flat.flat), ptr(flat.grad_flat), ptr(m), ptr(v), ptr(tab[0]), tab[1], tab[2], *hyper,
                       None, eng.rt.code, s)
    torch.cuda.synchronize()
    assert torch.equal(flat.flat, ref[0]) and torch.equal(m, ref[1]) and torch.equal(v, ref[2])
    changed = 0
    for k, t in imgs.items():
        assert torch.equal(t, ref[3][k]), f"image at {k:#x} differs"
        changed += int((t != img0[k]).sum())
    assert changed > 0

    # the device-hyper-parameter form (the captured step's) and the guard: a non-zero skip leaves everything put
    hd = torch.empty(8, dtype=torch.float32)
    L.mmseg_adamw_hyper(*hyper, hd.data_ptr())
    hd = hd.to(dev)
    flat.flat.copy_(p0), m.copy_(m0), v.copy_(v0)
    L.mmseg_adamw_pack_dev(ptr(flat.flat), ptr(flat.grad_flat), ptr(m), ptr(v), ptr(tab[0]), tab[1], tab[2], ptr(hd),
                           None, eng.rt.code, s)
    torch.cuda.synchronize()
    assert torch.equal(flat.flat, ref[0]) and torch.equal(m, ref[1]) and torch.equal(v, ref[2])
    skip = torch.ones(1, dtype=torch.float32, device=dev)
    before = (flat.flat.clone(), {k: t.clone() for k, t in imgs.items()})
    L.mmseg_adamw_pack_dev(ptr(flat.flat), ptr(flat.grad_flat), ptr(m), ptr(v), ptr(tab[0]), tab[1], tab[2], ptr(hd),
                           ptr(skip), eng.rt.code, s)
    torch.cuda.synchronize()
    assert torch.equal(flat.flat, before[0]) and all(torch.equal(t, before[1][k]) for k, t in imgs.items())


def _train(cfg, dev, model, steps, fused):
    torch.manual_seed(0)
    mdl = build_model(cfg)
    tr = Trainer(cfg, mdl)
    if not fused:
        tr.optimizer._pack_source = None
    batches = [_batch(dev, model, seed=k) for k in range(2)]
    losses = [tr.train_step(batches[i % 2], i) for i in range(steps)]
    torch.cuda.synchronize()
    return tr, losses, torch.cat([p.detach().reshape(-1) for p in mdl.parameters()]).clone()


@pytest.mark.parametrize("model", ["unet", "swin_unetr"])
def test_fused_step_equals_pack_every_forward(dev, model, monkeypatch):
    """Eager steps: FlatAdamW with the fused launch (the forward's pack skipped: Packer.fresh) against FlatAdamW
    without it (every forward packs): bitwise the same losses and parameters.  UNet3D also through the captured
    step (the graph's forward has no pack; the replay's AdamW keeps the images current)."""
    cfg = _cfg(model, "bfloat16")
    tr0, l0, p0 = _train(cfg, dev, model, 4, fused=False)
    tr1, l1, p1 = _train(cfg, dev, model, 4, fused=True)
    assert _engine(tr1).program.packer().fresh is not None
    assert l0 == l1 and torch.equal(p0, p1)
    if model == "unet":
        monkeypatch.setenv("MMSEG_STEP_GRAPH", "1")
        cfg["hardware"]["step_graph"] = True
        tr2, l2, p2 = _train(cfg, dev, model, 4, fused=True)
        assert len(tr2._graphs.graphs) == 2 and all(e["fused_pack"] for e in tr2._graphs.graphs.values())
        assert l0 == l2 and torch.equal(p0, p2)


def test_weights_changed_through_torch_are_repacked(dev):
    """After fused steps (images current, forward skips its pack), load_state_dict back to the initial weights:
    the next forward must see them (FlatParams.version changed), i.e. equal the initial model's output."""
    model = "unet"
    cfg = _cfg(model, "bfloat16")
    torch.manual_seed(0)
    mdl = build_model(cfg)
    tr = Trainer(cfg, mdl)
    x = _batch(dev, model)["image"]
    mdl.eval()
    with torch.no_grad():
        y0 = mdl(x).clone()
    sd0 = {k: t.clone() for k, t in mdl.state_dict().items()}
    mdl.train()
    for i in range(3):
        tr.train_step(_batch(dev, model, seed=i), i)
    mdl.eval()
    with torch.no_grad():
        y1 = mdl(x).clone()
    assert not torch.equal(y0, y1)
    mdl.load_state_dict(sd0)
    with torch.no_grad():
        y2 = mdl(x)
    assert torch.equal(y0, y2)
