"""CrossAttentionFusion / BidirectionalCrossAttention — mirror of the
reference's src/models/fusion/attention_fusion.py:77-216 on the HIP engine.

Same constructor arguments, parameter names (q_proj, k_proj, v_proj,
out_proj: nn.Conv3d(k=1); norm: nn.InstanceNorm3d) and forward signature
(query_features, key_value_features) -> [B, C, *spatial], so state dicts and
call sites carry over.  Forward and backward run as HIP launches
(engine/attention.py: every product on MFMA through mmseg_bgemm_nt); there is
no eager-PyTorch path: a CPU tensor raises.  `engine_dtype` selects fp32
(parity) or bf16 activation storage; parameters and gradients stay fp32.
Dropout on the attention matrix (:150) is only supported at p = 0 or in eval
mode (the reference's default and every config's value).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ...engine.attention import CrossAttentionEngine, FusionHeadEngine
from ...engine.runtime import Runtime

_NAMES = ("q", "k", "v", "o")


class _CrossAttentionFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, eng, q, kv, qw, qb, kw, kb, vw, vb, ow, ob):
        p = {"q_w": qw, "q_b": qb, "k_w": kw, "k_b": kb, "v_w": vw, "v_b": vb, "o_w": ow, "o_b": ob}
        y, st = eng.forward(q.contiguous(), kv.contiguous(), {k: v.detach().contiguous() for k, v in p.items()})
        ctx.eng, ctx.st, ctx.p = eng, st, {k: v.detach().contiguous() for k, v in p.items()}
        return y

    @staticmethod
    def backward(ctx, dy):
        eng, p = ctx.eng, ctx.p
        grads = {k: torch.empty_like(v) for k, v in p.items()}
        dq, dkv = eng.backward(dy.contiguous(), ctx.st, p, grads, accumulate=False)
        ctx.st = None
        return (None, dq, dkv) + tuple(grads[f"{n}_{t}"] for n in _NAMES for t in ("w", "b"))


class CrossAttentionFusion(nn.Module):
    """Reference attention_fusion.py:77-164."""

    def __init__(self, in_channels: int, num_heads: int = 4, dropout: float = 0.0,
                 engine_dtype: torch.dtype = torch.float32):
        super().__init__()
        self.in_channels = in_channels
        self.num_heads = num_heads
        self.head_dim = in_channels // num_heads
        assert in_channels % num_heads == 0, "in_channels must be divisible by num_heads"
        self.q_proj = nn.Conv3d(in_channels, in_channels, kernel_size=1)
        self.k_proj = nn.Conv3d(in_channels, in_channels, kernel_size=1)
        self.v_proj = nn.Conv3d(in_channels, in_channels, kernel_size=1)
        self.out_proj = nn.Conv3d(in_channels, in_channels, kernel_size=1)
        self.dropout = nn.Dropout(dropout)
        self.norm = nn.InstanceNorm3d(in_channels)
        self.out_channels = in_channels
        self.engine_dtype = engine_dtype
        self._eng = None

    def _engine(self, device: torch.device) -> CrossAttentionEngine:
        if self._eng is None or self._eng.rt.device != device:
            self._eng = CrossAttentionEngine(Runtime(device, self.engine_dtype), self.in_channels, self.num_heads)
        return self._eng

    def forward(self, query_features: torch.Tensor, key_value_features: torch.Tensor) -> torch.Tensor:
        if query_features.shape != key_value_features.shape:
            raise ValueError("query and key/value features must have the same shape")
        if self.training and self.dropout.p > 0:
            raise NotImplementedError("attention dropout > 0 is not on the engine (every config uses 0)")
        eng = self._engine(query_features.device)
        ps = [getattr(self, f"{n}_proj") for n in ("q", "k", "v", "out")]
        args = []
        for m in ps:
            args += [m.weight, m.bias]
        return _CrossAttentionFn.apply(eng, query_features.float(), key_value_features.float(), *args)


class BidirectionalCrossAttention(nn.Module):
    """Reference attention_fusion.py:167-216: both directions, then
    Conv3d(2C -> C, 1) + InstanceNorm3d + ReLU on the concatenation."""

    def __init__(self, in_channels: int, num_heads: int = 4, dropout: float = 0.0,
                 engine_dtype: torch.dtype = torch.float32):
        super().__init__()
        self.cross_attn_1to2 = CrossAttentionFusion(in_channels, num_heads, dropout, engine_dtype)
        self.cross_attn_2to1 = CrossAttentionFusion(in_channels, num_heads, dropout, engine_dtype)
        self.fusion = nn.Sequential(
            nn.Conv3d(in_channels * 2, in_channels, kernel_size=1),
            nn.InstanceNorm3d(in_channels),
            nn.ReLU(inplace=True),
        )
        self.out_channels = in_channels
        self._head = None

    def forward(self, features_1: torch.Tensor, features_2: torch.Tensor) -> torch.Tensor:
        a = self.cross_attn_1to2(features_1, features_2)
        b = self.cross_attn_2to1(features_2, features_1)
        if self._head is None or self._head.rt.device != a.device:
            self._head = FusionHeadEngine(Runtime(a.device, self.cross_attn_1to2.engine_dtype), a.shape[1])
        conv = self.fusion[0]
        return _FusionHeadFn.apply(self._head, a, b, conv.weight, conv.bias)


class _FusionHeadFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, eng, a, b, w, bias):
        w2 = w.detach().reshape(w.shape[0], -1).contiguous()
        y, st = eng.forward(a.contiguous(), b.contiguous(), w2, bias.detach().contiguous())
        ctx.eng, ctx.st, ctx.w2, ctx.wshape = eng, st, w2, w.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        gw = torch.empty(ctx.w2.shape, dtype=torch.float32, device=dy.device)
        gb = torch.empty(ctx.w2.shape[0], dtype=torch.float32, device=dy.device)
        da, db = ctx.eng.backward(dy.contiguous(), ctx.st, ctx.w2, gw, gb)
        ctx.st = None
        return None, da, db, gw.reshape(ctx.wshape), gb
