"""SwinUNETR entry of the model registry (reference swin_unetr.py:20-200) and the
MONAI window attention it is built from.

The reference wraps monai.networks.nets.SwinUNETR (swin_unetr.py:80-96); MONAI is
not installed in this image, so the arithmetic is parity-unpinned.
This round puts SwinUNETR's MFMA core on the engine: `WindowAttention` follows
MONAI 1.3's WindowAttention (monai/networks/nets/swin_unetr.py) — same
parameter names (qkv, proj, relative_position_bias_table, buffer
relative_position_index), same relative-position index construction, same
forward(x [B*nW, N, C], mask [nW, N, N] | None) — and runs forward + backward on
engine/attention.py:WindowAttentionEngine.  The full SwinUNETR network (patch
embedding, shifted-window stages, patch merging, UNETR decoder) is not on the
engine yet: building it raises, exactly like the reference does when MONAI is
missing (swin_unetr.py:71-72).
"""
from __future__ import annotations

from typing import Any, Dict, Sequence

import torch
import torch.nn as nn

from ...engine.attention import WindowAttentionEngine
from ...engine.runtime import Runtime


def relative_position_index(window_size: Sequence[int]) -> torch.Tensor:
    """MONAI WindowAttention.__init__ (3-D branch): index[n][m] into the
    (2w0-1)(2w1-1)(2w2-1)-row bias table for tokens n, m of one window."""
    w0, w1, w2 = window_size
    coords = torch.stack(torch.meshgrid(torch.arange(w0), torch.arange(w1), torch.arange(w2), indexing="ij"))
    flat = torch.flatten(coords, 1)
    rel = (flat[:, :, None] - flat[:, None, :]).permute(1, 2, 0).contiguous()
    rel[:, :, 0] += w0 - 1
    rel[:, :, 1] += w1 - 1
    rel[:, :, 2] += w2 - 1
    rel[:, :, 0] *= (2 * w1 - 1) * (2 * w2 - 1)
    rel[:, :, 1] *= 2 * w2 - 1
    return rel.sum(-1)


class _WindowAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mod, x, mask, qkv_w, qkv_b, proj_w, proj_b, table):
        p = {"qkv_w": qkv_w.detach().contiguous(), "proj_w": proj_w.detach().contiguous(),
             "proj_b": proj_b.detach().contiguous(), "table": table.detach().contiguous()}
        if qkv_b is not None:
            p["qkv_b"] = qkv_b.detach().contiguous()
        eng, index, csr = mod._device_state(x.device)
        y, st = eng.forward(x.float().contiguous(), None if mask is None else mask.float().contiguous(), p, index)
        ctx.mod, ctx.p, ctx.st, ctx.has_qkv_b = mod, p, st, qkv_b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        eng, _, csr = ctx.mod._device_state(dy.device)
        grads = {k: torch.empty_like(v) for k, v in ctx.p.items()}
        dx = eng.backward(dy.contiguous(), ctx.st, ctx.p, grads, csr)
        ctx.st = None
        return (None, dx, None, grads["qkv_w"], grads.get("qkv_b"), grads["proj_w"], grads["proj_b"],
                grads["table"])


class WindowAttention(nn.Module):
    """MONAI SwinUNETR WindowAttention on the engine (attention dropout / proj dropout must be 0, as in
    SwinUNETR's defaults)."""

    def __init__(self, dim: int, num_heads: int, window_size: Sequence[int], qkv_bias: bool = False,
                 attn_drop: float = 0.0, proj_drop: float = 0.0, engine_dtype: torch.dtype = torch.float32):
        super().__init__()
        if attn_drop or proj_drop:
            raise NotImplementedError("WindowAttention dropout is not on the engine (SwinUNETR uses 0)")
        self.dim, self.num_heads, self.window_size = dim, num_heads, tuple(window_size)
        self.scale = (dim // num_heads) ** -0.5
        w0, w1, w2 = self.window_size
        self.relative_position_bias_table = nn.Parameter(
            torch.zeros((2 * w0 - 1) * (2 * w1 - 1) * (2 * w2 - 1), num_heads))
        self.register_buffer("relative_position_index", relative_position_index(self.window_size))
        self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
        self.proj = nn.Linear(dim, dim)
        nn.init.trunc_normal_(self.relative_position_bias_table, std=0.02)
        self.engine_dtype = engine_dtype
        self._state = None

    def _device_state(self, device):
        if self._state is None or self._state[0].rt.device != device:
            N = self.relative_position_index.shape[0]
            idx = self.relative_position_index.reshape(-1).cpu().to(torch.int64)
            T = self.relative_position_bias_table.shape[0]
            order = torch.argsort(idx, stable=True)            # CSR of (n*N + m) per table row, ascending
            counts = torch.bincount(idx, minlength=T)
            offs = torch.zeros(T + 1, dtype=torch.int64)
            offs[1:] = torch.cumsum(counts, 0)
            csr = (offs.to(torch.int32).to(device), order.to(torch.int32).to(device), T)
            eng = WindowAttentionEngine(Runtime(device, self.engine_dtype), self.dim, self.num_heads)
            self._state = (eng, idx.to(torch.int32).to(device), csr)
            del N
        return self._state

    def forward(self, x: torch.Tensor, mask: torch.Tensor = None) -> torch.Tensor:
        n = x.shape[1]
        if n != self.relative_position_index.shape[0]:
            raise ValueError("the engine's window attention needs full windows (N = prod(window_size))")
        return _WindowAttnFn.apply(self, x, mask, self.qkv.weight, self.qkv.bias, self.proj.weight, self.proj.bias,
                                   self.relative_position_bias_table)


class SwinUNETR:  # pragma: no cover - the full network is not on the engine yet
    def __init__(self, *args, **kwargs):
        raise ImportError("the SwinUNETR network is not on the MI355X engine yet (SURVEY §8f rank 3; its window "
                          "attention is: models.backbones.swin_unetr.WindowAttention); use model.name 'unet' "
                          "or 'dual_encoder'")


def build_swin_unetr(config: Dict[str, Any]):
    return SwinUNETR()
