"""Pin the CPU oracle (oracle/mmseg_oracle.py) to the reference's own outputs
(golden fixtures captured from /root/reference by tests/golden/make_golden.py).
CPU only; these are what make the oracle trustworthy as the GPU parity checker."""
import numpy as np
import pytest
import torch

from oracle import mmseg_oracle as O
from tests.helpers import golden

torch.set_num_threads(min(8, torch.get_num_threads()))

TINY = {
    "unet_tiny": ("unet", 2, 3, None, O.dice_ce_loss),
    "dual_tiny_cross_attention": ("dual", 2, 3, "cross_attention", O.dice_ce_loss),
    "dual_tiny_concat": ("dual", 2, 3, "concat", O.dice_ce_loss),
    "dual_tiny_add": ("dual", 2, 3, "add", O.dice_ce_loss),
    "dual_tiny_attention": ("dual", 2, 3, "attention", O.dice_ce_loss),
    "dual_tiny_m3_tversky": ("dual", 3, 6, "cross_attention", O.tversky_loss),
}


def _setup(tag):
    kind, M, C, fz, lossf = TINY[tag]
    g = golden(tag)
    feats = list(g["features"])
    torch.manual_seed(int(g["seed"]))
    if kind == "unet":
        p = O.init_unet3d(M, C, feats)
        fwd = O.unet3d_forward
    else:
        p = O.init_dual_encoder(M, C, feats, fz)
        fwd = lambda pp, x: O.dual_encoder_forward(pp, x, fz)  # noqa: E731
    S, B, steps = int(g["S"]), int(g["B"]), int(g["steps"])
    gen = torch.Generator().manual_seed(int(g["seed"]) + 1)
    xs = torch.randn(steps + 1, B, M, S, S, S, generator=gen)
    ys = torch.randint(0, C, (steps + 1, B, S, S, S), generator=gen)
    return g, p, fwd, lossf, xs, ys


@pytest.mark.parametrize("tag", list(TINY))
def test_oracle_init_forward_grads(tag):
    g, p, fwd, lossf, xs, ys = _setup(tag)
    names = list(g["init_names"])
    assert list(p) == names
    assert np.array_equal(np.array([p[n].double().sum().item() for n in names]), g["init_sum"])
    pp = {k: v.clone().requires_grad_(True) for k, v in p.items()}
    out = fwd(pp, xs[0])
    loss = lossf(out, ys[0])
    loss.backward()
    flat = out.detach().reshape(-1)
    assert O.normwise_rel(flat[torch.from_numpy(g["sample_idx"])], torch.from_numpy(g["sample_logits"])) < 1e-5
    assert abs(loss.item() - float(g["loss"])) < 1e-6
    gn = np.array([pp[n].grad.double().norm().item() for n in names])
    live = gn > 1e-6 * gn.max()
    assert np.allclose(gn[live], g["grad_norm"][live], rtol=1e-4)


@pytest.mark.parametrize("tag", ["unet_tiny", "dual_tiny_attention"])
def test_oracle_trajectory(tag):
    g, p, fwd, lossf, xs, ys = _setup(tag)
    st = O.OracleStep(p, fwd, lossf, lr=1e-3, weight_decay=1e-5)
    tl = [st.step(xs[1 + i], ys[1 + i]) for i in range(int(g["steps"]))]
    assert np.allclose(tl, g["traj_losses"], rtol=0, atol=1e-6)


@pytest.mark.parametrize("C", [3, 6, 7])
def test_oracle_losses(C):
    g = golden("losses")
    logits = torch.from_numpy(g[f"logits_C{C}"])
    labels = torch.from_numpy(g[f"labels_C{C}"])
    cw = torch.from_numpy(g[f"cw_C{C}"])
    fns = {"dicece": O.dice_ce_loss, "dicece_w": lambda a, b: O.dice_ce_loss(a, b, 0.3, 0.7, cw),
           "dice": O.dice_loss, "dice_nobg": lambda a, b: O.dice_loss(a, b, include_background=False),
           "ce": O.ce_loss, "tversky": O.tversky_loss, "tversky_37": lambda a, b: O.tversky_loss(a, b, 0.3, 0.7),
           "focal": O.focal_loss, "focal_w": lambda a, b: O.focal_loss(a, b, cw)}
    for name, fn in fns.items():
        lg = logits.clone().requires_grad_(True)
        l = fn(lg, labels)
        l.backward()
        assert abs(l.item() - float(g[f"{name}_C{C}"])) < 1e-6, name
        assert O.normwise_rel(lg.grad, torch.from_numpy(g[f"{name}_C{C}_grad"])) < 1e-6, name


@pytest.mark.parametrize("C", [3, 6])
def test_oracle_dice_metric(C):
    g = golden("dice_metric")
    inter = np.zeros(C, np.int64)
    union = np.zeros(C, np.int64)
    for p, t in zip(g[f"pred_C{C}"], g[f"tgt_C{C}"]):
        i, u = O.dice_counts(p, t, C)
        inter += i
        union += u
    assert np.array_equal(inter, g[f"inter_C{C}"].astype(np.int64))
    assert np.array_equal(union, g[f"union_C{C}"].astype(np.int64))
    res = O.dice_metric_compute(inter, union)
    assert res["dice"] == float(g[f"dice_C{C}"])


def test_oracle_cross_attention_fusion():
    g = golden("cross_attention")
    p = {k[2:]: torch.from_numpy(g[k]) for k in g.files if k.startswith("p_")}
    q = torch.from_numpy(g["q"]).requires_grad_(True)
    kv = torch.from_numpy(g["kv"]).requires_grad_(True)
    out = O.cross_attention_fusion(p, "", q, kv, num_heads=4)
    assert O.normwise_rel(out, torch.from_numpy(g["out"])) < 1e-6
    (out * torch.from_numpy(g["cot"])).sum().backward()
    assert O.normwise_rel(q.grad, torch.from_numpy(g["dq"])) < 1e-5
    assert O.normwise_rel(kv.grad, torch.from_numpy(g["dkv"])) < 1e-5


def test_oracle_bidirectional_cross_attention():
    g = golden("bidirectional_attention")
    p = {k[2:]: torch.from_numpy(g[k]) for k in g.files if k.startswith("p_")}
    f1 = torch.from_numpy(g["f1"]).requires_grad_(True)
    f2 = torch.from_numpy(g["f2"]).requires_grad_(True)
    out = O.bidirectional_cross_attention(p, "", f1, f2, num_heads=4)
    assert O.normwise_rel(out, torch.from_numpy(g["out"])) < 1e-6
    (out * torch.from_numpy(g["cot"])).sum().backward()
    assert O.normwise_rel(f1.grad, torch.from_numpy(g["d1"])) < 1e-5
    assert O.normwise_rel(f2.grad, torch.from_numpy(g["d2"])) < 1e-5


def test_full_config_param_init_pinned():
    """full-size init checksums: the oracle's RNG order reproduces the reference's 22.6M / 36.7M params"""
    for tag, kind in (("full_unet_c2", "unet"), ("full_dual_c3", "dual")):
        g = golden(tag)
        torch.manual_seed(int(g["seed"]))
        p = (O.init_unet3d(2, 6, [32, 64, 128, 256, 512]) if kind == "unet"
             else O.init_dual_encoder(2, 6, [32, 64, 128, 256, 512], "cross_attention"))
        assert list(p) == list(g["param_names"])
        assert np.array_equal(np.array([v.double().sum().item() for v in p.values()]), g["param_sum"])


class _RecordPins(O.Pins):
    """Pins that record the oracle's own decisions (relu mask x > 0, MaxPool first argmax) while applying them."""

    def __init__(self):
        super().__init__([], [])

    def relu(self, x):
        self.relu_masks.append((x > 0).detach())
        return super().relu(x)

    def pool(self, x):
        N, C, D, H, W = x.shape
        win = x.detach().reshape(N, C, D // 2, 2, H // 2, 2, W // 2, 2).permute(0, 1, 2, 4, 6, 3, 5, 7)
        self.pool_codes.append(win.reshape(N, C, D // 2, H // 2, W // 2, 8).argmax(-1))
        return super().pool(x)


@pytest.mark.parametrize("kind", ["unet", "dual"])
def test_oracle_pins_reproduce_free_forward(kind):
    """Pinned with its own decisions, the oracle's forward and every gradient are bitwise the free oracle's:
    the pins only fix WHICH side of each kink a value is on, the arithmetic is unchanged."""
    feats = [8, 16, 32]
    torch.manual_seed(0)
    p = O.init_unet3d(2, 3, feats) if kind == "unet" else O.init_dual_encoder(2, 3, feats, "cross_attention")
    g = torch.Generator().manual_seed(1)
    x = torch.randn(2, 2, 16, 16, 16, generator=g, dtype=torch.float64)
    y = torch.randint(0, 3, (2, 16, 16, 16), generator=g)
    fwd = (lambda pp, xx, pins=None: O.unet3d_forward(pp, xx, 3, pins=pins)) if kind == "unet" else \
        (lambda pp, xx, pins=None: O.dual_encoder_forward(pp, xx, "cross_attention", 3, pins=pins))
    res = []
    rec = _RecordPins()
    for pins in (None, rec, "replay"):
        if pins == "replay":
            pins = O.Pins(rec.relu_masks, rec.pool_codes)
        pp = {k: v.double().requires_grad_(True) for k, v in p.items()}
        out = fwd(pp, x, pins)
        O.dice_ce_loss(out, y).backward()
        res.append((out.detach(), [pp[k].grad for k in p]))
    for out, grads in res[1:]:
        assert torch.equal(out, res[0][0])
        assert all(torch.equal(a, b) for a, b in zip(grads, res[0][1]))


def test_dice_envelope_fixture():
    """tests/golden/dice_heldout_envelope.npz (make_golden.py dice_heldout_envelope_case): the reference's free-running
    held-out Dice at 1/2/4/6 threads for both cases of test_dice_heldout_gpu.py, each a full trajectory of the stored
    length; the 8-thread run stored with the case itself lies inside the spread of the others widened by its width
    (the gate's construction is consistent with the data it was built from)."""
    import numpy as np
    from tests.helpers import golden
    e = golden("dice_heldout_envelope")
    assert list(e["threads"]) == [1, 2, 4, 6]
    for case, fix in (("c1", "dice_heldout_c1"), ("trained", "dice_heldout_trained")):
        g = golden(fix)
        d = e[f"{case}_f32_dice"]
        assert d.shape == (4,) and np.all((d > 0) & (d < 1))
        assert e[f"{case}_f32_train_losses"].shape == (4, int(g["K"]))
        lo, hi = d.min(), d.max()
        w = hi - lo
        assert lo - w <= float(g["f32_dice"]) <= hi + w
