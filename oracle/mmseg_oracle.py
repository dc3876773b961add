"""CPU oracle for the multimodal-organ-segmentation training hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product package imports this file;
only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` use it, and only as the checker / the timed CPU baseline.

It is a functional torch-CPU fp32 restatement of the reference's training
step (no reference code is imported or copied).  Each function cites the
reference file:line whose arithmetic it restates.  The restatement is pinned
against golden vectors captured from the reference itself in the build
container (``tests/golden/make_golden.py`` -> ``tests/golden/*.npz``); see
``tests/test_oracle_golden.py``.

Parameters are passed as a flat ``{name: tensor}`` dict using the
reference's backbone state-dict names (``init_conv.conv1.weight`` ...), so the
same dict can be loaded into the product model and compared key by key.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.nn.functional as F

Tensor = torch.Tensor
Params = Dict[str, Tensor]

IN_EPS = 1e-5  # nn.InstanceNorm3d default (reference unet.py:34-35)


# --------------------------------------------------------------------------
# parameter initialisation (reproduces the reference's RNG consumption order)
# --------------------------------------------------------------------------
def _conv3d_init(cin: int, cout: int, k: int) -> List[Tensor]:
    m = torch.nn.Conv3d(cin, cout, k, padding=k // 2)
    return [m.weight.detach().clone(), m.bias.detach().clone()]


def _convT_init(cin: int, cout: int) -> List[Tensor]:
    m = torch.nn.ConvTranspose3d(cin, cout, kernel_size=2, stride=2)
    return [m.weight.detach().clone(), m.bias.detach().clone()]


def _linear_init(fin: int, fout: int) -> List[Tensor]:
    m = torch.nn.Linear(fin, fout)
    return [m.weight.detach().clone(), m.bias.detach().clone()]


def _block_init(p: Params, prefix: str, cin: int, cout: int) -> None:
    # ConvBlock3D builds conv1 then conv2 (reference unet.py:26-27); the
    # InstanceNorm3d layers (affine=False) own no parameters.
    w, b = _conv3d_init(cin, cout, 3)
    p[prefix + "conv1.weight"], p[prefix + "conv1.bias"] = w, b
    w, b = _conv3d_init(cout, cout, 3)
    p[prefix + "conv2.weight"], p[prefix + "conv2.bias"] = w, b


def init_unet3d(in_channels: int, out_channels: int, features: Sequence[int]) -> Params:
    """Same construction order as reference unet.py:148-163."""
    p: Params = {}
    _block_init(p, "init_conv.", in_channels, features[0])
    for i in range(len(features) - 1):
        _block_init(p, f"encoders.{i}.conv.", features[i], features[i + 1])
    for j, i in enumerate(range(len(features) - 1, 0, -1)):
        w, b = _convT_init(features[i], features[i] // 2)
        p[f"decoders.{j}.up.weight"], p[f"decoders.{j}.up.bias"] = w, b
        _block_init(p, f"decoders.{j}.conv.", features[i], features[i - 1])
    w, b = _conv3d_init(features[0], out_channels, 1)
    p["out_conv.weight"], p["out_conv.bias"] = w, b
    return p


def init_dual_encoder(num_modalities: int, out_channels: int, features: Sequence[int],
                      fusion_type: str) -> Params:
    """Same construction order as reference dual_encoder.py:58-84."""
    p: Params = {}
    for m in range(num_modalities):
        _block_init(p, f"encoders.{m}.init_conv.", 1, features[0])
        for i in range(len(features) - 1):
            _block_init(p, f"encoders.{m}.blocks.{i}.conv.", features[i], features[i + 1])
    if fusion_type == "attention":
        for l, f in enumerate(features):
            mc = f * num_modalities
            w, b = _linear_init(mc, mc // 4)
            p[f"fusion_layers.{l}.attention.2.weight"], p[f"fusion_layers.{l}.attention.2.bias"] = w, b
            w, b = _linear_init(mc // 4, num_modalities)
            p[f"fusion_layers.{l}.attention.4.weight"], p[f"fusion_layers.{l}.attention.4.bias"] = w, b
    elif fusion_type == "concat":
        for l, f in enumerate(features):
            w, b = _conv3d_init(f * num_modalities, f, 1)
            p[f"fusion_proj.{l}.weight"], p[f"fusion_proj.{l}.bias"] = w, b
    for j, i in enumerate(range(len(features) - 1, 0, -1)):
        w, b = _convT_init(features[i], features[i] // 2)
        p[f"decoder.{j}.up.weight"], p[f"decoder.{j}.up.bias"] = w, b
        _block_init(p, f"decoder.{j}.conv.", features[i], features[i - 1])
    w, b = _conv3d_init(features[0], out_channels, 1)
    p["out_conv.weight"], p["out_conv.bias"] = w, b
    return p


# --------------------------------------------------------------------------
# kink pins (parity tests only)
# --------------------------------------------------------------------------
class Pins:
    """The piecewise-linear decisions of one forward, taken from the implementation under test: the ReLU mask
    of every InstanceNorm + ReLU (in forward order) and the argmax code t = 4 dz + 2 dy + dx of every MaxPool3d(2)
    window.  With them the oracle routes every gradient exactly as the implementation did, so an fp64 oracle
    and an fp32 implementation differ by rounding alone -- not by which side of a kink a value within rounding
    of it fell (at these decisions the true derivative jumps, so any two correct fp32 implementations disagree
    there by O(1) on those voxels)."""

    def __init__(self, relu_masks: List[Tensor], pool_codes: List[Tensor]):
        self.relu_masks, self.pool_codes = list(relu_masks), list(pool_codes)
        self.ri = self.pi = 0

    def relu(self, x: Tensor) -> Tensor:
        m = self.relu_masks[self.ri]
        self.ri += 1
        return x * m.to(x.dtype)

    def pool(self, x: Tensor) -> Tensor:
        code = self.pool_codes[self.pi]
        self.pi += 1
        N, C, D, H, W = x.shape
        win = x.reshape(N, C, D // 2, 2, H // 2, 2, W // 2, 2).permute(0, 1, 2, 4, 6, 3, 5, 7)
        win = win.reshape(N, C, D // 2, H // 2, W // 2, 8)
        return torch.gather(win, -1, code.long().unsqueeze(-1)).squeeze(-1)


def _relu(x: Tensor, pins: Optional[Pins]) -> Tensor:
    return torch.relu(x) if pins is None else pins.relu(x)


def _pool(x: Tensor, pins: Optional[Pins]) -> Tensor:
    return F.max_pool3d(x, 2) if pins is None else pins.pool(x)


# --------------------------------------------------------------------------
# forward restatements
# --------------------------------------------------------------------------
def conv_block(p: Params, prefix: str, x: Tensor, pins: Optional[Pins] = None) -> Tensor:
    """ConvBlock3D.forward: (conv3^3 -> InstanceNorm3d -> ReLU) x 2 (reference unet.py:53-60)."""
    for c in ("conv1", "conv2"):
        x = F.conv3d(x, p[prefix + c + ".weight"], p[prefix + c + ".bias"], padding=1)
        x = F.instance_norm(x, eps=IN_EPS)
        x = _relu(x, pins)
    return x


def up_block(p: Params, prefix: str, x: Tensor, skip: Tensor, pins: Optional[Pins] = None) -> Tensor:
    """UpBlock3D.forward: ConvTranspose3d(k2,s2) -> cat([up, skip]) -> ConvBlock (reference unet.py:104-113)."""
    x = F.conv_transpose3d(x, p[prefix + "up.weight"], p[prefix + "up.bias"], stride=2)
    if x.shape != skip.shape:  # dead for S divisible by 16 (reference unet.py:108-109)
        x = F.interpolate(x, size=skip.shape[2:], mode="trilinear", align_corners=True)
    return conv_block(p, prefix + "conv.", torch.cat([x, skip], dim=1), pins)


def unet3d_forward(p: Params, x: Tensor, n_levels: int = 5, pins: Optional[Pins] = None) -> Tensor:
    """UNet3D.forward (reference unet.py:165-200), dropout = identity."""
    x = conv_block(p, "init_conv.", x, pins)
    feats = [x]
    for i in range(n_levels - 1):
        x = conv_block(p, f"encoders.{i}.conv.", _pool(x, pins), pins)
        feats.append(x)
    skips = feats[:-1]
    for j, skip in enumerate(reversed(skips)):
        x = up_block(p, f"decoders.{j}.", x, skip, pins)
    return F.conv3d(x, p["out_conv.weight"], p["out_conv.bias"])


def cross_modal_attention(p: Params, prefix: str, stacked: Tensor) -> Tensor:
    """CrossModalAttention.forward (reference dual_encoder.py:235-254): SE gate over modalities."""
    B, M, C = stacked.shape[:3]
    pooled = stacked.reshape(B, M * C, -1).mean(dim=-1)                      # AdaptiveAvgPool3d(1)+Flatten
    h = torch.relu(F.linear(pooled, p[prefix + "attention.2.weight"], p[prefix + "attention.2.bias"]))
    w = torch.softmax(F.linear(h, p[prefix + "attention.4.weight"], p[prefix + "attention.4.bias"]), dim=1)
    return (stacked * w.view(B, M, 1, 1, 1, 1)).sum(dim=1)


def fuse_level(p: Params, fusion_type: str, level: int, feats: List[Tensor]) -> Tensor:
    """DualEncoder._fuse_features (reference dual_encoder.py:167-199)."""
    if fusion_type == "concat":
        return F.conv3d(torch.cat(feats, dim=1), p[f"fusion_proj.{level}.weight"], p[f"fusion_proj.{level}.bias"])
    if fusion_type == "add":
        out = feats[0]
        for f in feats[1:]:
            out = out + f
        return out
    if fusion_type == "attention":
        return cross_modal_attention(p, f"fusion_layers.{level}.", torch.stack(feats, dim=1))
    # every other string (incl. "cross_attention", "early", "late") -> mean (dual_encoder.py:193-195)
    return torch.stack(feats).mean(dim=0)


def dual_encoder_forward(p: Params, x: Tensor, fusion_type: str, n_levels: int = 5,
                         pins: Optional[Pins] = None) -> Tensor:
    """DualEncoder.forward (reference dual_encoder.py:112-165), dropout = identity."""
    M = x.shape[1]
    per_mod = []
    for m in range(M):
        f = conv_block(p, f"encoders.{m}.init_conv.", x[:, m:m + 1], pins)
        fl = [f]
        for i in range(n_levels - 1):
            f = conv_block(p, f"encoders.{m}.blocks.{i}.conv.", _pool(f, pins), pins)
            fl.append(f)
        per_mod.append(fl)
    fused = [fuse_level(p, fusion_type, l, [pm[l] for pm in per_mod]) for l in range(n_levels)]
    y = fused[-1]
    for j, skip in enumerate(reversed(fused[:-1])):
        y = up_block(p, f"decoder.{j}.", y, skip, pins)
    return F.conv3d(y, p["out_conv.weight"], p["out_conv.bias"])


def cross_attention_fusion(p: Params, prefix: str, q_feat: Tensor, kv_feat: Tensor, num_heads: int) -> Tensor:
    """CrossAttentionFusion.forward (reference attention_fusion.py:120-164), dropout = identity."""
    B, C = q_feat.shape[:2]
    hd = C // num_heads
    conv = lambda n, t: F.conv3d(t, p[prefix + n + ".weight"], p[prefix + n + ".bias"])
    Q = conv("q_proj", q_feat).reshape(B, num_heads, hd, -1)
    K = conv("k_proj", kv_feat).reshape(B, num_heads, hd, -1)
    V = conv("v_proj", kv_feat).reshape(B, num_heads, hd, -1)
    attn = torch.softmax(torch.einsum("bhdn,bhdm->bhnm", Q, K) * hd ** -0.5, dim=-1)
    out = torch.einsum("bhnm,bhdm->bhdn", attn, V).reshape(q_feat.shape)
    return F.instance_norm(q_feat + conv("out_proj", out), eps=IN_EPS)


def bidirectional_cross_attention(p: Params, prefix: str, f1: Tensor, f2: Tensor, num_heads: int) -> Tensor:
    """BidirectionalCrossAttention.forward (reference attention_fusion.py:202-216): both directions, then
    Conv3d(2C -> C, 1) + InstanceNorm3d + ReLU (:196-200)."""
    a = cross_attention_fusion(p, prefix + "cross_attn_1to2.", f1, f2, num_heads)
    b = cross_attention_fusion(p, prefix + "cross_attn_2to1.", f2, f1, num_heads)
    z = F.conv3d(torch.cat([a, b], dim=1), p[prefix + "fusion.0.weight"], p[prefix + "fusion.0.bias"])
    return F.relu(F.instance_norm(z, eps=IN_EPS))


def window_attention(p: Params, prefix: str, x: Tensor, mask, num_heads: int, index: Tensor) -> Tensor:
    """MONAI 1.3 SwinUNETR WindowAttention.forward (monai/networks/nets/swin_unetr.py; the reference builds it
    through swin_unetr.py:80-96) restated: qkv linear, q * scale, q @ k^T, + relative-position bias, (+ mask of
    window b % nW), softmax, @ v, proj.  MONAI is absent: parity vs MONAI itself is unpinned."""
    b, n, c = x.shape
    hd = c // num_heads
    qkv = F.linear(x, p[prefix + "qkv.weight"], p.get(prefix + "qkv.bias"))
    qkv = qkv.reshape(b, n, 3, num_heads, hd).permute(2, 0, 3, 1, 4)
    q, k, v = qkv[0] * hd ** -0.5, qkv[1], qkv[2]
    attn = q @ k.transpose(-2, -1)
    table = p[prefix + "relative_position_bias_table"]
    bias = table[index[:n, :n].reshape(-1)].reshape(n, n, -1).permute(2, 0, 1)
    attn = attn + bias.unsqueeze(0)
    if mask is not None:
        nw = mask.shape[0]
        attn = attn.view(b // nw, nw, num_heads, n, n) + mask.unsqueeze(1).unsqueeze(0)
        attn = attn.view(-1, num_heads, n, n)
    attn = torch.softmax(attn, dim=-1)
    out = (attn @ v).transpose(1, 2).reshape(b, n, c)
    return F.linear(out, p[prefix + "proj.weight"], p[prefix + "proj.bias"])


# --------------------------------------------------------------------------
# sliding-window inference (reference trainer.py:370-395 -> MONAI 1.3
# monai.inferers.sliding_window_inference, constant blending; MONAI is absent
# here, so this restates its published algorithm: parity vs MONAI unpinned)
# --------------------------------------------------------------------------
def sliding_window_inference(inputs: Tensor, roi_size, sw_batch_size: int, predictor, overlap: float = 0.25) -> Tensor:
    """CPU restatement: pad to the roi (zeros, symmetric), scan interval int(roi * (1 - overlap)) (roi when the
    padded size equals the roi), dense_patch_slices starts (last window clamped to the end), windows image-major
    in meshgrid 'ij' order, batched sw_batch_size at a time, output += pred, count_map += 1, output / count_map,
    crop.  `predictor` receives each window batch on its own device; results are accumulated on the CPU."""
    import math
    N, M = inputs.shape[:2]
    size = list(inputs.shape[2:])
    roi = [r if r > 0 else s for r, s in zip(roi_size, size)]
    pad = []
    for k in range(len(size) - 1, -1, -1):          # F.pad order: last dim first
        diff = max(roi[k] - size[k], 0)
        pad += [diff // 2, diff - diff // 2]
    x = F.pad(inputs.float().cpu(), pad, mode="constant", value=0.0)
    psize = list(x.shape[2:])
    interval = []
    for r, s in zip(roi, psize):
        interval.append(r if r == s else max(int(r * (1 - overlap)), 1))
    starts = []
    for d in range(3):
        num = int(math.ceil(float(psize[d]) / interval[d]))
        scan = next((i for i in range(num) if i * interval[d] + roi[d] >= psize[d]), None)
        cnt = scan + 1 if scan is not None else 1
        starts.append([i * interval[d] - max(i * interval[d] + roi[d] - psize[d], 0) for i in range(cnt)])
    slices = [(a, b, c) for a in starts[0] for b in starts[1] for c in starts[2]]
    wins = [(n, s_) for n in range(N) for s_ in slices]
    out, count = None, None
    dev = inputs.device
    for b0 in range(0, len(wins), sw_batch_size):
        chunk = wins[b0:b0 + sw_batch_size]
        batch = torch.stack([x[n, :, a:a + roi[0], b:b + roi[1], c:c + roi[2]] for n, (a, b, c) in chunk])
        pred = predictor(batch.to(dev))
        pred = (pred[0] if isinstance(pred, (tuple, list)) else pred).float().cpu()
        if out is None:
            out = torch.zeros(N, pred.shape[1], *psize)
            count = torch.zeros(N, 1, *psize)
        for k, (n, (a, b, c)) in enumerate(chunk):
            out[n, :, a:a + roi[0], b:b + roi[1], c:c + roi[2]] += pred[k]
            count[n, :, a:a + roi[0], b:b + roi[1], c:c + roi[2]] += 1.0
    out = out / count
    lo = [pad[2 * (2 - d)] for d in range(3)]
    return out[:, :, lo[0]:lo[0] + size[0], lo[1]:lo[1] + size[1], lo[2]:lo[2] + size[2]]


# --------------------------------------------------------------------------
# losses / metric
# --------------------------------------------------------------------------
def _softmax_onehot(pred: Tensor, target: Tensor):
    C = pred.shape[1]
    prob = torch.softmax(pred, dim=1).flatten(2)
    onehot = F.one_hot(target, C).movedim(-1, 1).to(pred.dtype).flatten(2)
    return prob, onehot


def dice_loss(pred: Tensor, target: Tensor, smooth: float = 1.0, include_background: bool = True) -> Tensor:
    """DiceLoss.forward (reference losses.py:39-80), reduction mean."""
    prob, onehot = _softmax_onehot(pred, target)
    if not include_background:
        prob, onehot = prob[:, 1:], onehot[:, 1:]
    inter = (prob * onehot).sum(-1)
    union = prob.sum(-1) + onehot.sum(-1)
    return (1.0 - (2.0 * inter + smooth) / (union + smooth)).mean()


def ce_loss(pred: Tensor, target: Tensor, class_weights: Optional[Tensor] = None) -> Tensor:
    """nn.CrossEntropyLoss(weight) mean reduction (reference losses.py:214)."""
    return F.cross_entropy(pred, target, weight=class_weights)


def dice_ce_loss(pred: Tensor, target: Tensor, dice_weight: float = 0.5, ce_weight: float = 0.5,
                 class_weights: Optional[Tensor] = None) -> Tensor:
    """DiceCELoss.forward (reference losses.py:216-228)."""
    return dice_weight * dice_loss(pred, target) + ce_weight * ce_loss(pred, target, class_weights)


def tversky_loss(pred: Tensor, target: Tensor, alpha: float = 0.5, beta: float = 0.5, smooth: float = 1.0) -> Tensor:
    """TverskyLoss.forward (reference losses.py:160-185)."""
    prob, onehot = _softmax_onehot(pred, target)
    tp = (prob * onehot).sum(-1)
    fp = (prob * (1 - onehot)).sum(-1)
    fn = ((1 - prob) * onehot).sum(-1)
    return (1.0 - (tp + smooth) / (tp + alpha * fp + beta * fn + smooth)).mean()


def focal_loss(pred: Tensor, target: Tensor, alpha: Optional[Tensor] = None, gamma: float = 2.0) -> Tensor:
    """FocalLoss.forward (reference losses.py:107-125): class-weighted voxel CE, (1 - exp(-ce))^gamma * ce, mean."""
    ce = F.cross_entropy(pred, target, weight=alpha, reduction="none")
    pt = torch.exp(-ce)
    return ((1 - pt) ** gamma * ce).mean()


def dice_counts(pred_idx: np.ndarray, target_idx: np.ndarray, num_classes: int):
    """Per-class integer intersection/union counts of DiceMetric.update (reference metrics.py:42-67)."""
    p = np.asarray(pred_idx).reshape(-1)
    t = np.asarray(target_idx).reshape(-1)
    inter = np.bincount(t[p == t], minlength=num_classes)[:num_classes].astype(np.int64)
    union = (np.bincount(p, minlength=num_classes)[:num_classes]
             + np.bincount(t, minlength=num_classes)[:num_classes]).astype(np.int64)
    return inter, union


def dice_metric_compute(inter: np.ndarray, union: np.ndarray, include_background: bool = False) -> Dict[str, object]:
    """DiceMetric.compute (reference metrics.py:69-88); accumulators are fp32 tensors in the reference."""
    inter_t = torch.tensor(inter, dtype=torch.float32)
    union_t = torch.tensor(union, dtype=torch.float32)
    dpc = (2.0 * inter_t + 1e-5) / (union_t + 1e-5)
    start = 0 if include_background else 1
    return {"dice": dpc[start:].mean().item(), "dice_per_class": dpc.tolist()}


# --------------------------------------------------------------------------
# training step (Trainer._train_epoch per-batch body, reference trainer.py:250-258)
# --------------------------------------------------------------------------
class OracleStep:
    """fp32 CPU train step: forward -> loss -> backward -> AdamW (accumulation_steps = 1)."""

    def __init__(self, params: Params, forward, loss_fn, lr=1e-4, weight_decay=1e-5, betas=(0.9, 0.999)):
        self.params = {k: v.detach().clone().requires_grad_(True) for k, v in params.items()}
        self.forward = forward
        self.loss_fn = loss_fn
        self.opt = torch.optim.AdamW(list(self.params.values()), lr=lr, weight_decay=weight_decay, betas=betas)

    def step(self, x: Tensor, y: Tensor) -> float:
        self.opt.zero_grad()
        out = self.forward(self.params, x)
        loss = self.loss_fn(out, y)
        loss.backward()
        self.opt.step()
        return float(loss.item())

    def grads(self) -> Params:
        return {k: v.grad.detach().clone() for k, v in self.params.items()}


def normwise_rel(a: Tensor, b: Tensor) -> float:
    """max|a-b| / max|b| — the 'normwise' relative error the parity bar is stated in."""
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    den = b.abs().max().item()
    return (a - b).abs().max().item() / (den if den > 0 else 1.0)
