"""CPU oracle for SwinUNETR (config c4) — TEST INFRASTRUCTURE ONLY.

Nothing in the product package imports this file; only ``tests/`` use it, as
the checker.  The reference wraps ``monai.networks.nets.SwinUNETR``
(reference src/models/backbones/swin_unetr.py:80-96, built by
build_swin_unetr swin_unetr.py:180-200 with downsample="merging",
use_v2=False, normalize=True, qkv_bias=True, mlp_ratio 4, window 7, patch 2).
MONAI is not installed and not on disk, so this file restates the
MONAI 1.3 SwinUNETR forward from its published architecture in functional
torch-CPU fp32.  **Parity vs MONAI itself is unpinned**: the engine is checked
against this restatement only.  The functions follow their inputs' device: the
128^3 c4 backward check evaluates them in fp64 on the GPU (tests only).

Parameters are a flat ``{name: tensor}`` dict keyed by the MONAI state-dict
names below a prefix (``swinViT.layers1.0.blocks.0.attn.qkv.weight`` ...), so
the product module's ``state_dict()`` feeds it directly.

MONAI quirks kept on purpose (both are what MONAI 1.3 computes):
  * the legacy PatchMerging ("merging") concatenates the 8 half-resolution
    sub-grids in the order (0,0,0) (1,0,0) (0,1,0) (0,0,1) (1,0,1) (0,1,0)
    (0,0,1) (1,1,1) (z,y,x parities) — (0,1,0) and (0,0,1) twice, (1,1,0)
    and (0,1,1) never;
  * a window smaller than 7 (a stage whose grid is <= 7 per side) indexes the
    7^3 relative-position table with relative_position_index[:n, :n].
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional

import numpy as np
import torch
import torch.nn.functional as F

from .mmseg_oracle import window_attention

Tensor = torch.Tensor
Params = Dict[str, Tensor]

LN_EPS = 1e-5
IN_EPS = 1e-5
LRELU_SLOPE = 0.01
MERGE_ORDER = ((0, 0, 0), (1, 0, 0), (0, 1, 0), (0, 0, 1), (1, 0, 1), (0, 1, 0), (0, 0, 1), (1, 1, 1))


def dropout_keep(seed: int, n: int, p: float) -> np.ndarray:
    """Keep mask of the engine's counter-hash dropout (csrc/swin.hip dropout_kernel) for hash indices 0..n-1:
    splitmix64(seed + h * 0x9E3779B97F4A7C15) >> 32 >= p * 2^32.  MONAI draws its masks from torch's RNG, so
    mask-level parity with the reference is undefined; this restates the engine's generator so the tests can
    check that every site applies it (and its backward) where MONAI applies nn.Dropout."""
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + np.arange(n, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
    t = float(np.float32(p)) * 4294967296.0      # p reaches the kernel as a C float
    thr = 0xFFFFFFFF if t >= 4294967295.0 else int(t)
    return (z >> np.uint64(32)) >= np.uint64(thr)


def make_drop(p: float, seeds: Dict[str, object]) -> Callable[[Tensor, str], Tensor]:
    """drop(t, site) for the oracle: t * keep / (1 - p) with the engine's mask of that site, where t is the
    tensor in MONAI's layout at the site (pos_drop: NCDHW patch embedding; proj: [B*nW, N, C] windows; drop1 /
    drop2: [b, d, h, w, c] token grids) and the hash index is t's flat index."""
    scale = torch.tensor(1.0 / (1.0 - float(np.float32(p))), dtype=torch.float32)

    def drop(t: Tensor, site: str) -> Tensor:
        if site == "pos":
            seed = seeds["pos"]
        else:
            pre, which = site.rsplit(".", 1)
            seed = seeds[pre + "."][{"proj": 0, "drop1": 1, "drop2": 2}[which]]
        keep = torch.from_numpy(dropout_keep(int(seed), t.numel(), p)).view(t.shape).to(t.device)
        return torch.where(keep, t * scale.to(t.dtype), torch.zeros((), dtype=t.dtype))

    return drop


def relative_position_index(window) -> Tensor:
    """MONAI WindowAttention.__init__ (3-D): index[n][m] of token pair (n, m) into the
    (2w0-1)(2w1-1)(2w2-1)-row relative-position bias table."""
    w0, w1, w2 = window
    coords = torch.stack(torch.meshgrid(torch.arange(w0), torch.arange(w1), torch.arange(w2), indexing="ij"))
    flat = torch.flatten(coords, 1)
    rel = (flat[:, :, None] - flat[:, None, :]).permute(1, 2, 0).contiguous()
    rel[:, :, 0] += w0 - 1
    rel[:, :, 1] += w1 - 1
    rel[:, :, 2] += w2 - 1
    rel[:, :, 0] *= (2 * w1 - 1) * (2 * w2 - 1)
    rel[:, :, 1] *= 2 * w2 - 1
    return rel.sum(-1)


def get_window_size(x_size, window_size, shift_size):
    """MONAI get_window_size: a side no larger than the window uses the whole side and no shift."""
    ws, ss = list(window_size), list(shift_size)
    for i in range(len(x_size)):
        if x_size[i] <= window_size[i]:
            ws[i] = x_size[i]
            ss[i] = 0
    return tuple(ws), tuple(ss)


def window_partition(x: Tensor, ws) -> Tensor:
    b, d, h, w, c = x.shape
    x = x.view(b, d // ws[0], ws[0], h // ws[1], ws[1], w // ws[2], ws[2], c)
    return x.permute(0, 1, 3, 5, 2, 4, 6, 7).contiguous().view(-1, ws[0] * ws[1] * ws[2], c)


def window_reverse(windows: Tensor, ws, dims) -> Tensor:
    b, d, h, w = dims
    x = windows.view(b, d // ws[0], h // ws[1], w // ws[2], ws[0], ws[1], ws[2], -1)
    return x.permute(0, 1, 4, 2, 5, 3, 6, 7).contiguous().view(b, d, h, w, -1)


def compute_mask(dims, ws, ss) -> Tensor:
    """MONAI compute_mask (3-D): region labels of the shifted grid, -100 between different regions."""
    cnt = 0
    d, h, w = dims
    img = torch.zeros((1, d, h, w, 1))
    for a in (slice(-ws[0]), slice(-ws[0], -ss[0]), slice(-ss[0], None)):
        for b in (slice(-ws[1]), slice(-ws[1], -ss[1]), slice(-ss[1], None)):
            for c in (slice(-ws[2]), slice(-ws[2], -ss[2]), slice(-ss[2], None)):
                img[:, a, b, c, :] = cnt
                cnt += 1
    mw = window_partition(img, ws).squeeze(-1)
    m = mw.unsqueeze(1) - mw.unsqueeze(2)
    return m.masked_fill(m != 0, float(-100.0)).masked_fill(m == 0, float(0.0))


def swin_block(p: Params, pre: str, x: Tensor, mask: Tensor, window, shift, heads: int, index: Tensor,
               drop: Optional[Callable] = None) -> Tensor:
    """SwinTransformerBlock.forward (part1: LN, pad, roll, window attention (+ proj_drop), reverse, unroll, crop;
    residual; part2: LN, MLP(linear1, GELU, drop1, linear2, drop2); residual).  x [b, d, h, w, c]."""
    b, d, h, w, c = x.shape
    ws, ss = get_window_size((d, h, w), window, shift)
    shortcut = x
    y = F.layer_norm(x, (c,), p[pre + "norm1.weight"], p[pre + "norm1.bias"], LN_EPS)
    pd, ph, pw = [(ws[i] - s % ws[i]) % ws[i] for i, s in enumerate((d, h, w))]
    y = F.pad(y, (0, 0, 0, pw, 0, ph, 0, pd))
    _, dp, hp, wp, _ = y.shape
    if any(i > 0 for i in ss):
        y = torch.roll(y, shifts=(-ss[0], -ss[1], -ss[2]), dims=(1, 2, 3))
        m = mask
    else:
        m = None
    xw = window_partition(y, ws)
    aw = window_attention(p, pre + "attn.", xw, m, heads, index)
    if drop is not None:
        aw = drop(aw.reshape(-1, ws[0] * ws[1] * ws[2], c), pre + "proj")
    y = window_reverse(aw.view(-1, ws[0] * ws[1] * ws[2], c), ws, (b, dp, hp, wp))
    if any(i > 0 for i in ss):
        y = torch.roll(y, shifts=ss, dims=(1, 2, 3))
    y = y[:, :d, :h, :w, :]
    x = shortcut + y
    z = F.layer_norm(x, (c,), p[pre + "norm2.weight"], p[pre + "norm2.bias"], LN_EPS)
    z = F.linear(z, p[pre + "mlp.linear1.weight"], p[pre + "mlp.linear1.bias"])
    z = F.gelu(z)
    if drop is not None:
        z = drop(z, pre + "drop1")
    z = F.linear(z, p[pre + "mlp.linear2.weight"], p[pre + "mlp.linear2.bias"])
    if drop is not None:
        z = drop(z, pre + "drop2")
    return x + z


def patch_merging(p: Params, pre: str, x: Tensor) -> Tensor:
    """Legacy PatchMerging (downsample="merging"): pad odd sides, gather 8 sub-grids (MERGE_ORDER), LN(8c),
    Linear(8c -> 2c, no bias)."""
    b, d, h, w, c = x.shape
    if d % 2 or h % 2 or w % 2:
        x = F.pad(x, (0, 0, 0, w % 2, 0, h % 2, 0, d % 2))
    x = torch.cat([x[:, i::2, j::2, k::2, :] for i, j, k in MERGE_ORDER], -1)
    x = F.layer_norm(x, (8 * c,), p[pre + "norm.weight"], p[pre + "norm.bias"], LN_EPS)
    return F.linear(x, p[pre + "reduction.weight"])


def basic_layer(p: Params, pre: str, x: Tensor, depth: int, heads: int, window, index: Tensor,
                drop: Optional[Callable] = None) -> Tensor:
    """BasicLayer.forward: x [b, c, d, h, w] -> blocks (even: no shift, odd: shift window//2) -> PatchMerging."""
    b, c, d, h, w = x.shape
    shift_full = tuple(i // 2 for i in window)
    ws, ss = get_window_size((d, h, w), window, shift_full)
    x = x.permute(0, 2, 3, 4, 1)
    dp, hp, wp = [-(-s // ws[i]) * ws[i] for i, s in enumerate((d, h, w))]
    mask = compute_mask((dp, hp, wp), ws, ss).to(x.device)
    for i in range(depth):
        x = swin_block(p, f"{pre}blocks.{i}.", x, mask, window, (0, 0, 0) if i % 2 == 0 else shift_full, heads,
                       index, drop)
    x = patch_merging(p, pre + "downsample.", x)
    return x.permute(0, 4, 1, 2, 3)


def proj_out(x: Tensor, normalize: bool = True) -> Tensor:
    """SwinTransformer.proj_out: layer_norm over channels without affine (normalize=True)."""
    if not normalize:
        return x
    c = x.shape[1]
    return F.layer_norm(x.permute(0, 2, 3, 4, 1), (c,), eps=LN_EPS).permute(0, 4, 1, 2, 3)


def swin_transformer(p: Params, pre: str, x: Tensor, depths, heads, window, index: Tensor,
                     normalize: bool = True, drop: Optional[Callable] = None) -> List[Tensor]:
    """SwinTransformer.forward: patch_embed (Conv3d k2 s2), pos_drop, proj_out of every stage's output."""
    x0 = F.conv3d(x, p[pre + "patch_embed.proj.weight"], p[pre + "patch_embed.proj.bias"], stride=2)
    if drop is not None:
        x0 = drop(x0, "pos")
    outs = [proj_out(x0, normalize)]
    h = x0
    for i in range(4):
        h = basic_layer(p, f"{pre}layers{i + 1}.0.", h, depths[i], heads[i], window, index, drop)
        outs.append(proj_out(h, normalize))
    return outs


class LReluPins:
    """The LeakyReLU decisions (pre-activation > 0, in forward order) of the implementation under test, so that
    the oracle routes 1 or LRELU_SLOPE of every voxel's gradient exactly as it did (test infrastructure; the
    same idea as mmseg_oracle.Pins)."""

    def __init__(self, masks):
        self.masks, self.i = list(masks), 0

    def take(self) -> Tensor:
        m = self.masks[self.i]
        self.i += 1
        return m


def _lrelu(x: Tensor, pins: Optional[LReluPins] = None) -> Tensor:
    if pins is None:
        return F.leaky_relu(x, LRELU_SLOPE)
    m = pins.take().to(device=x.device, dtype=torch.bool)
    return x * torch.where(m, torch.ones((), dtype=x.dtype), torch.full((), LRELU_SLOPE, dtype=x.dtype))


def unet_res_block(p: Params, pre: str, x: Tensor, pins: Optional[LReluPins] = None) -> Tensor:
    """UnetResBlock: conv1 -> IN -> LeakyReLU(0.01) -> conv2 -> IN, + residual (conv3 1x1 -> IN when the channel
    count changes), LeakyReLU.  Convs without bias, IN without affine."""
    out = F.conv3d(x, p[pre + "conv1.conv.weight"], padding=1)
    out = _lrelu(F.instance_norm(out, eps=IN_EPS), pins)
    out = F.conv3d(out, p[pre + "conv2.conv.weight"], padding=1)
    out = F.instance_norm(out, eps=IN_EPS)
    res = x
    if pre + "conv3.conv.weight" in p:
        res = F.instance_norm(F.conv3d(x, p[pre + "conv3.conv.weight"]), eps=IN_EPS)
    return _lrelu(out + res, pins)


def unetr_up_block(p: Params, pre: str, x: Tensor, skip: Tensor, pins: Optional[LReluPins] = None) -> Tensor:
    """UnetrUpBlock: ConvTranspose3d(k2 s2, no bias) -> cat([up, skip]) -> UnetResBlock."""
    up = F.conv_transpose3d(x, p[pre + "transp_conv.conv.weight"], stride=2)
    return unet_res_block(p, pre + "conv_block.", torch.cat([up, skip], 1), pins)


def swin_unetr_forward(p: Params, x: Tensor, depths=(2, 2, 2, 2), heads=(3, 6, 12, 24), window=(7, 7, 7),
                       normalize: bool = True, prefix: str = "", drop: Optional[Callable] = None,
                       pins: Optional[LReluPins] = None) -> Tensor:
    """MONAI SwinUNETR.forward: x [b, M, S^3] -> logits [b, C, S^3].  drop: the drop_rate sites in training
    mode (make_drop), None = eval / drop_rate 0.  pins: the LeakyReLU decisions of the ten residual blocks, in
    this call order (encoder1/2/3/4/10, decoder5..1), two per block."""
    index = relative_position_index(window).to(x.device)
    hs = swin_transformer(p, prefix + "swinViT.", x, depths, heads, window, index, normalize, drop)
    enc0 = unet_res_block(p, prefix + "encoder1.layer.", x, pins)
    enc1 = unet_res_block(p, prefix + "encoder2.layer.", hs[0], pins)
    enc2 = unet_res_block(p, prefix + "encoder3.layer.", hs[1], pins)
    enc3 = unet_res_block(p, prefix + "encoder4.layer.", hs[2], pins)
    dec4 = unet_res_block(p, prefix + "encoder10.layer.", hs[4], pins)
    dec3 = unetr_up_block(p, prefix + "decoder5.", dec4, hs[3], pins)
    dec2 = unetr_up_block(p, prefix + "decoder4.", dec3, enc3, pins)
    dec1 = unetr_up_block(p, prefix + "decoder3.", dec2, enc2, pins)
    dec0 = unetr_up_block(p, prefix + "decoder2.", dec1, enc1, pins)
    out = unetr_up_block(p, prefix + "decoder1.", dec0, enc0, pins)
    return F.conv3d(out, p[prefix + "out.conv.conv.weight"], p[prefix + "out.conv.conv.bias"])
