"""SwinUNETR (MONAI 1.3 architecture, reached from the reference's
swin_unetr.py:80-96) as a whole-network HIP program over the flat parameter
arena — config c4's model.

MONAI is absent: the arithmetic follows oracle/swin_oracle.py,
the restatement the tests hold this program to (parity vs MONAI unpinned).

Layout.  Swin stages run on channels-last token grids [N, d, h, w, C]
(the engine's NDHWC, ld = C).  The UNETR side (residual conv blocks,
transposed convs, head) runs on NDHWC buffers whose channel stride is padded
to 8 x a power of two (48 -> 64, 96 -> 128, ...): the implicit-GEMM conv
kernels split K into power-of-two channel groups, and the padded channels
meet zero weights (pack modes 0 / 6 / 7), so they only need to be finite —
every such buffer is zero-initialised once when the shape is planned.

Kernels: LayerNorm / GELU / window partition+roll / reverse+roll+residual /
patch-merging gather (csrc/swin.hip), window attention core (relative-position
bias, shifted-window mask; engine/attention.py on mmseg_bgemm_nt MFMA),
token linears as 1x1 implicit GEMMs (mmseg_conv_gemm MODE_POINT) with
split-K weight gradients (mmseg_wgrad + mmseg_wgrad_reduce), UNETR convs on
the same conv kernels as UNet3D, InstanceNorm statistics / backward from
norm_pool.hip, the LeakyReLU residual tail (mmseg_res_apply / _lrelu_bwd).
"""
from __future__ import annotations

import math
import os
from typing import Optional, Tuple

import numpy as np
import torch
import torch.nn as nn

from .._lib import ptr
from .attention import WindowAttentionEngine
from .layers import (MODE_POINT, Conv3, ConvT2, Head, Packer, _col_tile, _gemm_ksplit, _gemm_name, _io_bytes,
                     _own_part, _wgrad_ksplit)
from .profiler import TIMER
from .runtime import Act, FlatParams, Runtime, round_up

LN_EPS = 1e-5
IN_EPS = 1e-5
SLOPE = 0.01   # MONAI UnetResBlock LeakyReLU negative_slope


def cpad(c: int) -> int:
    """Channel stride of a UNETR-side buffer: 8 x the next power of two."""
    return max(8, 1 << int(math.ceil(math.log2(c))))


def window_size_for(dims, window, shift):
    """MONAI get_window_size."""
    ws, ss = list(window), list(shift)
    for i, d in enumerate(dims):
        if d <= window[i]:
            ws[i], ss[i] = d, 0
    return tuple(ws), tuple(ss)


def shift_regions(dims_p, ws, ss) -> np.ndarray:
    """Region label of every token of every window [nW, N] (MONAI compute_mask's img_mask, partitioned)."""
    img = np.zeros(dims_p, dtype=np.float32)
    cnt = 0
    for a in (slice(-ws[0]), slice(-ws[0], -ss[0]), slice(-ss[0], None)):
        for b in (slice(-ws[1]), slice(-ws[1], -ss[1]), slice(-ss[1], None)):
            for c in (slice(-ws[2]), slice(-ws[2], -ss[2]), slice(-ss[2], None)):
                img[a, b, c] = cnt
                cnt += 1
    d, h, w = dims_p
    t = img.reshape(d // ws[0], ws[0], h // ws[1], ws[1], w // ws[2], ws[2]).transpose(0, 2, 4, 1, 3, 5)
    return t.reshape(-1, ws[0] * ws[1] * ws[2])


def shift_mask(dims_p, ws, ss) -> np.ndarray:
    """MONAI compute_mask (3-D) on the padded grid: [nW, N, N] with -100 between tokens of different shifted
    regions (host-side plan, once per shape)."""
    img = np.zeros(dims_p, dtype=np.float32)
    cnt = 0
    for a in (slice(-ws[0]), slice(-ws[0], -ss[0]), slice(-ss[0], None)):
        for b in (slice(-ws[1]), slice(-ws[1], -ss[1]), slice(-ss[1], None)):
            for c in (slice(-ws[2]), slice(-ws[2], -ss[2]), slice(-ss[2], None)):
                img[a, b, c] = cnt
                cnt += 1
    d, h, w = dims_p
    t = img.reshape(d // ws[0], ws[0], h // ws[1], ws[1], w // ws[2], ws[2]).transpose(0, 2, 4, 1, 3, 5)
    t = t.reshape(-1, ws[0] * ws[1] * ws[2])
    m = t[:, None, :] - t[:, :, None]
    return np.where(m != 0, np.float32(-100.0), np.float32(0.0)).astype(np.float32)


def _res_fuse() -> bool:
    """The residual sums folded into their producers (mmseg_conv_gemm_res, mmseg_lrelu_bwd_in_part); MMSEG_RES_FUSE=0
    keeps the separate passes (bitwise the same results)."""
    return os.environ.get("MMSEG_RES_FUSE", "1") != "0"


class Lin:
    """Token linear y[M][Co] = x[M][Cip] W^T (+ b) as a 1x1 implicit GEMM (MODE_POINT), weight [Co][Ci...]
    (trailing dims flattened: the PatchEmbed kernel [Co][Cin][2][2][2] is a [Co][8 Cin] linear over the
    patchified input).  Backward: split-K weight (+ bias) gradient into the arena, data gradient GEMM."""

    def __init__(self, rt: Runtime, weight: nn.Parameter, bias: Optional[nn.Parameter], flat: FlatParams,
                 cin_pad: Optional[int] = None, need_dgrad: bool = True):
        self.rt, self.w, self.b, self.flat = rt, weight, bias, flat
        self.Co = weight.shape[0]
        self.Ci = weight.numel() // self.Co
        self.Cip = cin_pad or self.Ci
        if self.Co % 8 or self.Cip % 8:
            raise ValueError("token linear: channel counts must be multiples of 8")
        self.KG, self.Cpad = self.Cip // 8, _col_tile(self.Co)
        self.KGp = round_up(self.KG, 4)
        self.wf = torch.zeros(self.KGp * self.Cpad * 8, dtype=rt.dtype, device=rt.device)
        self.need_dgrad = need_dgrad
        if need_dgrad:
            self.KGd, self.Cpad_d = self.Co // 8, _col_tile(self.Ci)
            self.KGdp = round_up(self.KGd, 4)
            self.wd = torch.zeros(self.KGdp * self.Cpad_d * 8, dtype=rt.dtype, device=rt.device)

    def descs(self):
        d = [(ptr(self.w), ptr(self.wf), 2, self.Co, self.Ci, self.Cip, self.KG, self.KGp, self.Cpad)]
        if self.need_dgrad:
            d.append((ptr(self.w), ptr(self.wd), 3, self.Co, self.Ci, self.Ci, self.KGd, self.KGdp, self.Cpad_d))
        return d

    def fwd_gelu(self, x: torch.Tensor, ldx: int, M: int, h: torch.Tensor, g: torch.Tensor) -> None:
        """h = x W^T + b and g = gelu(h) (MLPBlock linear1 + GELU; dense rows of Co): from the GEMM's epilogue
        (mmseg_conv_gemm_gelu) when it runs without split-K, else the GEMM + mmseg_gelu_fwd -- bitwise the same."""
        L = self.rt.lib
        if _gemm_ksplit(M, self.Co, self.KG) == 1 and _res_fuse():
            with TIMER.region(_gemm_name(self.rt, 0, "point"), flops=2.0 * M * self.Ci * self.Co,
                              nbytes=_io_bytes(self.rt, M, self.Cip, 2 * self.Co, self.Ci * self.Co)):
                L.mmseg_conv_gemm_gelu(ptr(x), ldx, ptr(self.wf), ptr(self.b), ptr(h), self.Co, None, ptr(g), 1, M,
                                       self.Co, self.Cpad, self.KG, self.rt.code, self.rt.stream)
            return
        self.fwd(x, ldx, M, h, self.Co)
        L.mmseg_gelu_fwd(ptr(h), ptr(g), M * self.Co, self.rt.code, self.rt.stream)

    def fwd(self, x: torch.Tensor, ldx: int, M: int, y: torch.Tensor, ldy: int, res: Optional[torch.Tensor] = None,
            ncols: Optional[int] = None):
        """res (pitch ldy, may be y): y = res + x W^T (+ b), from the GEMM's epilogue when it runs without split-K
        (mmseg_conv_gemm_res), else through a temporary and mmseg_add -- bitwise the same.  ncols (> Co, bias-free,
        <= the packed column tile): the GEMM also writes the zero columns [Co, ncols) of its zero-padded weights, so
        y's padded rows are written whole (Act.wcols) and one column tile covers 48 real columns."""
        L = self.rt.lib
        nc = self.Co if ncols is None else ncols
        if nc != self.Co and (self.b is not None or nc > self.Cpad or nc % 8 or res is not None):
            raise ValueError(f"token linear: {nc} output columns need a bias-free layer within its packed tile")
        ks = _gemm_ksplit(M, nc, self.KG)
        fuse = res is not None and ks == 1 and _res_fuse()
        out = y if res is None or fuse else torch.empty(M * ldy, dtype=self.rt.dtype, device=self.rt.device)
        ws = self.rt.ws(ks * M * nc) if ks > 1 else None
        with TIMER.region(_gemm_name(self.rt, 0, "point"), flops=2.0 * M * self.Ci * self.Co,
                          nbytes=_io_bytes(self.rt, M, self.Cip, self.Co, self.Ci * self.Co)):
            if fuse:
                L.mmseg_conv_gemm_res(ptr(x), ldx, ptr(self.wf), ptr(self.b), ptr(res), ldy, ptr(y), ldy, M, self.Co,
                                      self.Cpad, self.KG, self.rt.code, self.rt.stream)
            else:
                L.mmseg_conv_gemm(ptr(x), ldx, ptr(self.wf), ptr(self.b), ptr(out), ldy, ptr(ws), MODE_POINT, M,
                                  nc, self.Cpad, self.KG, 0, 1, 1, 1, ks, self.rt.code, self.rt.stream)
        if res is not None and not fuse:
            if ldy != self.Co:
                raise ValueError("token linear with a residual: dense rows only on the unfused path")
            L.mmseg_add(ptr(res), ptr(out), ptr(y), M * ldy, self.rt.code, self.rt.stream)

    def bwd(self, x: torch.Tensor, ldx: int, dy: torch.Tensor, lddy: int, M: int, dx: Optional[torch.Tensor],
            lddx: int, accumulate: bool, dx_add: bool = False, dx_cols: Optional[int] = None,
            gelu_h: Optional[torch.Tensor] = None):
        """dx_add: dx += the data gradient (a residual branch's; the GEMM's epilogue adds it, mmseg_conv_gemm_res,
        when it runs without split-K), instead of dx := it.  dx_cols: as fwd's ncols for dx (zero columns
        [Ci, dx_cols) from the zero-padded data-gradient image: whole-row writes).  gelu_h: dx := (dy W) * gelu'(gelu_h)
        (the data gradient through the GELU that produced this layer's input; dense rows), in the GEMM's epilogue
        when it runs without split-K, else the GEMM + mmseg_gelu_bwd -- bitwise the same."""
        L, s, code = self.rt.lib, self.rt.stream, self.rt.code
        ks = L.mmseg_wgrad_splits(M, _wgrad_ksplit(self.Co, self.Cip, M))
        defer = self.rt.defer_wred(self.flat)
        nfl = ks * self.Co * self.Cip + ks * self.Co + 4
        part = _own_part(self, self.rt, nfl) if defer else self.rt.ws(nfl)
        bpart = part.data_ptr() + round_up(ks * self.Co * self.Cip, 4) * 4 if self.b is not None else None
        with TIMER.region(_gemm_name(self.rt, 0, "point"), flops=2.0 * M * self.Ci * self.Co,
                          nbytes=_io_bytes(self.rt, M, self.Cip, self.Co, self.Ci * self.Co, 4)):
            L.mmseg_wgrad(ptr(dy), lddy, ptr(x), ldx, ptr(part), bpart, MODE_POINT, self.Co, self.Cip, 0, M, 1, 1, 1,
                          ks, code, s)
        (L.mmseg_wgrad_reduce_defer if defer else L.mmseg_wgrad_reduce)(
            ptr(part), ptr(self.flat.grad(self.w)), bpart, ptr(self.flat.grad(self.b)) if self.b is not None else None,
            self.Co, self.Cip, ks, self.Cip, self.Ci, 1, int(accumulate), s)
        self.flat.mark(*[p for p in (self.w, self.b) if p is not None])
        if dx is not None:
            ncd = self.Ci if dx_cols is None else dx_cols
            if ncd != self.Ci and (ncd > self.Cpad_d or ncd % 8):
                raise ValueError(f"token linear: {ncd} data-gradient columns exceed the packed tile {self.Cpad_d}")
            kd = _gemm_ksplit(M, ncd, self.KGd)
            if dx_add and (kd > 1 or not _res_fuse()):
                raise ValueError("Lin.bwd(dx_add): the residual epilogue needs the unsplit GEMM")
            ws = self.rt.ws(kd * M * ncd) if kd > 1 else None
            gelu_fused = gelu_h is not None and kd == 1 and _res_fuse()
            with TIMER.region(_gemm_name(self.rt, 0, "point"), flops=2.0 * M * self.Ci * self.Co,
                              nbytes=_io_bytes(self.rt, M, self.Co, self.Ci, self.Ci * self.Co)):
                if gelu_fused:
                    if dx_add or ncd != self.Ci or lddx != self.Ci:
                        raise ValueError("Lin.bwd(gelu_h): dense data gradient only")
                    L.mmseg_conv_gemm_gelu(ptr(dy), lddy, ptr(self.wd), None, ptr(dx), lddx, ptr(gelu_h), None, 2, M,
                                           self.Ci, self.Cpad_d, self.KGd, code, s)
                elif dx_add:
                    L.mmseg_conv_gemm_res(ptr(dy), lddy, ptr(self.wd), None, ptr(dx), lddx, ptr(dx), lddx, M, ncd,
                                          self.Cpad_d, self.KGd, code, s)
                else:
                    L.mmseg_conv_gemm(ptr(dy), lddy, ptr(self.wd), None, ptr(dx), lddx, ptr(ws), MODE_POINT, M,
                                      ncd, self.Cpad_d, self.KGd, 0, 1, 1, 1, kd, code, s)
            if gelu_h is not None and not gelu_fused:
                L.mmseg_gelu_bwd(ptr(gelu_h), ptr(dx), ptr(dx), M * self.Ci, code, s)

    def dgrad_splits(self, M: int, ncols: Optional[int] = None) -> int:
        return _gemm_ksplit(M, self.Ci if ncols is None else ncols, self.KGd)


class LN:
    """nn.LayerNorm(C) over token rows (gamma / beta None: proj_out's affine-free layer_norm)."""

    def __init__(self, rt: Runtime, norm: Optional[nn.LayerNorm], C: int, flat: FlatParams):
        self.rt, self.norm, self.C, self.flat = rt, norm, C, flat

    def fwd(self, x, ldx, rows, y, ldy):
        mean = torch.empty(rows, dtype=torch.float32, device=self.rt.device)
        rstd = torch.empty(rows, dtype=torch.float32, device=self.rt.device)
        g = self.norm.weight if self.norm is not None else None
        b = self.norm.bias if self.norm is not None else None
        self.rt.lib.mmseg_layernorm_fwd(ptr(x), ldx, ptr(y), ldy, rows, self.C, ptr(g), ptr(b), LN_EPS, ptr(mean),
                                        ptr(rstd), self.rt.code, self.rt.stream)
        return mean, rstd

    def bwd(self, x, ldx, stats, dy, lddy, dx, lddx, rows, add_dx: bool, accumulate: bool):
        L = self.rt.lib
        mean, rstd = stats
        if self.norm is not None:
            ws = self.rt.ws(L.mmseg_layernorm_bwd_ws_floats(rows, self.C))
            L.mmseg_layernorm_bwd(ptr(x), ldx, ptr(dy), lddy, ptr(dx), lddx, rows, self.C, ptr(self.norm.weight),
                                  ptr(mean), ptr(rstd), int(add_dx), ptr(self.flat.grad(self.norm.weight)),
                                  ptr(self.flat.grad(self.norm.bias)), int(accumulate), ptr(ws), self.rt.code,
                                  self.rt.stream)
            self.flat.mark(self.norm.weight, self.norm.bias)
        else:
            L.mmseg_layernorm_bwd(ptr(x), ldx, ptr(dy), lddy, ptr(dx), lddx, rows, self.C, None, ptr(mean), ptr(rstd),
                                  int(add_dx), None, None, 0, None, self.rt.code, self.rt.stream)


class Drop:
    """nn.Dropout(drop_rate) at MONAI SwinUNETR's sites (pos_drop, proj_drop, MLP drop1 / drop2) on the
    counter-hash kernel mmseg_dropout: each forward draws one seed per site from torch's CPU generator
    (so torch.manual_seed fixes the masks) and the backward re-applies the same call to the gradient."""

    def __init__(self, rt: Runtime, p: float):
        self.rt, self.p = rt, float(p)

    @staticmethod
    def seed() -> int:
        return int(torch.randint(0, 2 ** 62, (1,)).item())

    def __call__(self, src: torch.Tensor, dst: torch.Tensor, rows: int, C: int, seed: int, V: int = 1,
                 ncdhw: bool = False):
        self.rt.lib.mmseg_dropout(ptr(src), ptr(dst), rows, C, V, int(ncdhw), self.p, seed, self.rt.code,
                                  self.rt.stream)


class SwinBlockProg:
    """SwinTransformerBlock: x + attn(windows(LN1(x))), then + MLP(LN2(.))."""

    def __init__(self, rt: Runtime, blk: nn.Module, flat: FlatParams, dim: int, heads: int, shifted: bool):
        self.rt, self.blk, self.flat, self.C, self.heads, self.shifted = rt, blk, flat, dim, heads, shifted
        a = blk.attn
        self.ln1 = LN(rt, blk.norm1, dim, flat)
        self.ln2 = LN(rt, blk.norm2, dim, flat)
        self.qkv = Lin(rt, a.qkv.weight, a.qkv.bias, flat)
        self.proj = Lin(rt, a.proj.weight, a.proj.bias, flat)
        self.fc1 = Lin(rt, blk.mlp.linear1.weight, blk.mlp.linear1.bias, flat)
        self.fc2 = Lin(rt, blk.mlp.linear2.weight, blk.mlp.linear2.bias, flat)
        self.core = WindowAttentionEngine(rt, dim, heads)
        self.table = a.relative_position_bias_table

    def descs(self):
        return self.qkv.descs() + self.proj.descs() + self.fc1.descs() + self.fc2.descs()

    def _table_t(self) -> torch.Tensor:
        """The bias table [T][heads] transposed to [heads][T] (one contiguous row per head for the kernels)."""
        T, h = self.table.shape
        out = torch.empty(h * T, dtype=torch.float32, device=self.rt.device)
        self.rt.lib.mmseg_transpose(ptr(self.table), 0, 0, h, 0, ptr(out), 0, 0, T, 0, 1, 1, T, h, self.rt.stream)
        return out

    def _fused(self, Nw: int) -> bool:
        """The fused window-attention kernels (csrc/winattn.hip): bf16 storage, head_dim 8 / 16, <= 352
        tokens per window (MMSEG_WINATTN=0: the batched-GEMM path)."""
        import os
        return (self.rt.code == 1 and self.core.hd in (8, 16) and Nw <= 352
                and os.environ.get("MMSEG_WINATTN", "1") != "0")

    def _empty(self, n):
        return torch.empty(int(n), dtype=self.rt.dtype, device=self.rt.device)

    def fwd(self, x: torch.Tensor, geo, drop: Optional[Drop] = None) -> Tuple[torch.Tensor, dict]:
        """x [N*d*h*w][C] (storage dtype) -> (out, saved state).  drop: the block's three dropout sites
        (training with drop_rate > 0), else None."""
        rt, L, s, code, C = self.rt, self.rt.lib, self.rt.stream, self.rt.code, self.C
        seeds = (Drop.seed(), Drop.seed(), Drop.seed()) if drop is not None else None
        N, d, h, w = geo["grid"]
        ws, (dp, hp, wp) = geo["ws"], geo["padded"]
        sh = geo["ss"] if self.shifted else (0, 0, 0)
        M = N * d * h * w
        Nw = ws[0] * ws[1] * ws[2]
        B = N * (dp // ws[0]) * (hp // ws[1]) * (wp // ws[2])
        Mw = B * Nw
        ln1 = self._empty(M * C)
        st1 = self.ln1.fwd(x, C, M, ln1, C)
        xw = self._empty(Mw * C)
        L.mmseg_window_partition(ptr(ln1), C, N, d, h, w, C, *ws, *sh, dp, hp, wp, ptr(xw), code, s)
        del ln1
        qkv = self._empty(Mw * 3 * C)
        self.qkv.fwd(xw, C, Mw, qkv, 3 * C)
        mask = geo["mask"] if any(sh) else None
        fused = self._fused(Nw)
        if fused:
            O = self._empty(Mw * C)
            P = torch.empty(L.mmseg_winattn_lse_floats(B, self.heads), dtype=torch.float32, device=rt.device)
            region = geo["region"] if any(sh) else None
            nw = region.shape[0] if region is not None else 0
            w0, w1, w2 = geo["window"]
            tabT = self._table_t()
            # algorithmic work: S = Q K^T and O = P V, 2 * 2 * Nw^2 * hd per (window, head); bytes: q, k, v in, O out
            with TIMER.region(lambda: L.mmseg_last_kernel().decode(), flops=4.0 * B * Nw * Nw * C,
                              nbytes=2.0 * Mw * 4 * C):
                L.mmseg_winattn_fwd(ptr(qkv), B, Nw, C, self.heads, ptr(tabT), self.table.shape[0], w0, w1, w2,
                                    ptr(region), nw, self.core.scale, ptr(O), ptr(P), s)
        else:
            O, P = self.core.core_fwd(qkv, B, Nw, mask, self.table, geo["index"])
        aw = self._empty(Mw * C)
        self.proj.fwd(O, C, Mw, aw, C)
        if seeds:                         # WindowAttention.proj_drop over the [B*nW, N, C] windows
            drop(aw, aw, Mw, C, seeds[0])
        xm = self._empty(M * C)
        L.mmseg_window_reverse(ptr(aw), N, d, h, w, C, *ws, *sh, dp, hp, wp, ptr(x), C, ptr(xm), C, code, s)
        del aw
        ln2 = self._empty(M * C)
        st2 = self.ln2.fwd(xm, C, M, ln2, C)
        hdim = self.fc1.Co
        hbuf = self._empty(M * hdim)
        g = self._empty(M * hdim)
        self.fc1.fwd_gelu(ln2, C, M, hbuf, g)          # h = linear1(.), g = GELU(h)
        if seeds:                         # MLPBlock drop1 (after the activation)
            drop(g, g, M, hdim, seeds[1])
        out = self._empty(M * C)
        if seeds:
            z = self._empty(M * C)
            self.fc2.fwd(g, hdim, M, z, C)
            drop(z, z, M, C, seeds[2])    # MLPBlock drop2 (after linear2)
            L.mmseg_add(ptr(xm), ptr(z), ptr(out), M * C, code, s)
        else:
            self.fc2.fwd(g, hdim, M, out, C, res=xm)     # out = xm + linear2(.)
        st = dict(x=x, st1=st1, xw=xw, qkv=qkv, O=O, P=P, xm=xm, st2=st2, ln2=ln2, h=hbuf, g=g, B=B, Nw=Nw, Mw=Mw,
                  M=M, sh=sh, fused=fused, drop=drop, seeds=seeds)
        return out, st

    def bwd(self, dout: torch.Tensor, st: dict, geo, accumulate: bool) -> torch.Tensor:
        """dout [M][C] -> dx, written over dout's buffer."""
        rt, L, s, code, C = self.rt, self.rt.lib, self.rt.stream, self.rt.code, self.C
        N, d, h, w = geo["grid"]
        ws, (dp, hp, wp) = geo["ws"], geo["padded"]
        M, Mw, B, Nw, sh = st["M"], st["Mw"], st["B"], st["Nw"], st["sh"]
        hdim = self.fc1.Co
        drop, seeds = st["drop"], st["seeds"]
        dz = dout
        if seeds:
            dz = self._empty(M * C)
            drop(dout, dz, M, C, seeds[2])
        dg = self._empty(M * hdim)
        if seeds:
            self.fc2.bwd(st["g"], hdim, dz, C, M, dg, hdim, accumulate)
            drop(dg, dg, M, hdim, seeds[1])
            L.mmseg_gelu_bwd(ptr(st["h"]), ptr(dg), ptr(dg), M * hdim, code, s)
        else:                             # d(linear1 output) = (dz W2) * GELU'(h)
            self.fc2.bwd(st["g"], hdim, dz, C, M, dg, hdim, accumulate, gelu_h=st["h"])
        del dz
        dln2 = self._empty(M * C)
        self.fc1.bwd(st["ln2"], C, dg, hdim, M, dln2, C, accumulate)
        del dg
        self.ln2.bwd(st["xm"], C, st["st2"], dln2, C, dout, C, M, True, accumulate)   # dout := d xm
        daw = self._empty(Mw * C)
        L.mmseg_window_partition(ptr(dout), C, N, d, h, w, C, *ws, *sh, dp, hp, wp, ptr(daw), code, s)
        if seeds:
            drop(daw, daw, Mw, C, seeds[0])
        dO = self._empty(Mw * C)
        self.proj.bwd(st["O"], C, daw, C, Mw, dO, C, accumulate)
        del daw
        if st["fused"]:
            dqkv = self._empty(Mw * 3 * C)
            ldn = (Nw + 7) // 8 * 8
            region = geo["region"] if any(sh) else None
            nw = region.shape[0] if region is not None else 0
            w0, w1, w2 = geo["window"]
            dB = torch.empty(self.heads * Nw * Nw, dtype=torch.float32, device=rt.device)
            offs, pairs, T = geo["csr"]
            # many windows: the score gradient summed over window groups on chip (fp32, mmseg_winattn_bwd_sum),
            # so the bias-table gradient folds a few group sums instead of every window's bf16 dS
            ng = L.mmseg_winattn_sum_groups(B, Nw, self.heads)
            # algorithmic backward work: dP = dO V^T, dV = P^T dO, dK = dS^T Q (the key pass, 3 x 2 Nw^2 hd) and
            # dQ = dS K (the query pass, 2 Nw^2 hd); the recomputed scores are not counted
            kv_w = ("winattn_bwd_kv2_kernel", 6.0 * B * Nw * Nw * C, 2.0 * Mw * 8 * C)
            if ng > 0:
                dsum = torch.empty(ng * self.heads * Nw * ldn, dtype=torch.float32, device=rt.device)
                with TIMER.region(*kv_w, more=[("winattn_bwd_qb2_kernel", 2.0 * B * Nw * Nw * C, 2.0 * Mw * 7 * C)]):
                    L.mmseg_winattn_bwd_sum(ptr(st["qkv"]), ptr(st["O"]), ptr(dO), ptr(st["P"]), B, Nw, C,
                                            self.heads, ptr(self._table_t()), self.table.shape[0], w0, w1, w2,
                                            ptr(region), nw, self.core.scale, ptr(dqkv), ptr(dsum), ldn, s)
                L.mmseg_relpos_table_grad(ptr(dsum), ldn, ng, self.heads, Nw, ptr(dB), ptr(offs), ptr(pairs), T,
                                          ptr(self.flat.grad(self.table)), int(accumulate), 0, s)   # dsum: fp32
                del dsum
            else:
                dS = self._empty(B * self.heads * Nw * ldn)
                with TIMER.region(*kv_w, more=[("winattn_bwd_q2_kernel", 2.0 * B * Nw * Nw * C, 2.0 * Mw * 7 * C)]):
                    L.mmseg_winattn_bwd(ptr(st["qkv"]), ptr(st["O"]), ptr(dO), ptr(st["P"]), B, Nw, C, self.heads,
                                        ptr(self._table_t()), self.table.shape[0], w0, w1, w2, ptr(region), nw,
                                        self.core.scale, ptr(dqkv), ptr(dS), ldn, s)
                L.mmseg_relpos_table_grad(ptr(dS), ldn, B, self.heads, Nw, ptr(dB), ptr(offs), ptr(pairs), T,
                                          ptr(self.flat.grad(self.table)), int(accumulate), code, s)
                del dS
        else:
            dqkv = self.core.core_bwd(dO, st["qkv"], st["P"], B, Nw, self.flat.grad(self.table), geo["csr"],
                                      accumulate)
        self.flat.mark(self.table)
        del dO
        dxw = self._empty(Mw * C)
        self.qkv.bwd(st["xw"], C, dqkv, 3 * C, Mw, dxw, C, accumulate)
        del dqkv
        dln1 = self._empty(M * C)
        L.mmseg_window_reverse(ptr(dxw), N, d, h, w, C, *ws, *sh, dp, hp, wp, None, 0, ptr(dln1), C, code, s)
        self.ln1.bwd(st["x"], C, st["st1"], dln1, C, dout, C, M, True, accumulate)    # dout := d x
        return dout


class SwinStageProg:
    """BasicLayer: depth blocks (odd ones shifted) + legacy PatchMerging (gather, LN(8C), Linear 8C -> 2C)."""

    def __init__(self, rt: Runtime, layer: nn.Module, flat: FlatParams, dim: int, heads: int, window):
        self.rt, self.dim, self.window = rt, dim, tuple(window)
        self.blocks = [SwinBlockProg(rt, b, flat, dim, heads, i % 2 == 1) for i, b in enumerate(layer.blocks)]
        self.index_full = layer.blocks[0].attn.relative_position_index
        self.table_rows = layer.blocks[0].attn.relative_position_bias_table.shape[0]
        self.mnorm = LN(rt, layer.downsample.norm, 8 * dim, flat)
        self.red = Lin(rt, layer.downsample.reduction.weight, None, flat)
        self.geo = None

    def descs(self):
        d = []
        for b in self.blocks:
            d += b.descs()
        return d + self.red.descs()

    def setup(self, N, d, h, w):
        dev = self.rt.device
        shift_full = tuple(i // 2 for i in self.window)
        ws, ss = window_size_for((d, h, w), self.window, shift_full)
        padded = tuple(-(-s // ws[i]) * ws[i] for i, s in enumerate((d, h, w)))
        Nw = ws[0] * ws[1] * ws[2]
        idx = self.index_full[:Nw, :Nw].reshape(-1).cpu().to(torch.int64)
        order = torch.argsort(idx, stable=True)
        counts = torch.bincount(idx, minlength=self.table_rows)
        offs = torch.zeros(self.table_rows + 1, dtype=torch.int64)
        offs[1:] = torch.cumsum(counts, 0)
        mask = torch.from_numpy(shift_mask(padded, ws, ss)).to(dev) if any(ss) else None
        region = (torch.from_numpy(shift_regions(padded, ws, ss).astype(np.uint8)).to(dev) if any(ss) else None)
        self.geo = dict(grid=(N, d, h, w), ws=ws, ss=ss, padded=padded, mask=mask, region=region,
                        window=self.window,
                        index=idx.to(torch.int32).to(dev),
                        csr=(offs.to(torch.int32).to(dev), order.to(torch.int32).to(dev), self.table_rows))
        self.out_dims = tuple((s + 1) // 2 for s in (d, h, w))

    def fwd(self, x: torch.Tensor, drop: Optional[Drop] = None):
        rt, L, C = self.rt, self.rt.lib, self.dim
        N, d, h, w = self.geo["grid"]
        self.saved = []
        for b in self.blocks:
            x, st = b.fwd(x, self.geo, drop)
            self.saved.append(st)
        d2, h2, w2 = self.out_dims
        M2 = N * d2 * h2 * w2
        cat = torch.empty(M2 * 8 * C, dtype=rt.dtype, device=rt.device)
        L.mmseg_merge_gather(ptr(x), C, N, d, h, w, C, ptr(cat), rt.code, rt.stream)
        lnm = torch.empty_like(cat)
        stm = self.mnorm.fwd(cat, 8 * C, M2, lnm, 8 * C)
        y = torch.empty(M2 * 2 * C, dtype=rt.dtype, device=rt.device)
        self.red.fwd(lnm, 8 * C, M2, y, 2 * C)
        self.msaved = (cat, lnm, stm, M2)
        return y

    def bwd(self, dy: torch.Tensor, accumulate: bool) -> torch.Tensor:
        rt, L, C = self.rt, self.rt.lib, self.dim
        N, d, h, w = self.geo["grid"]
        d2, h2, w2 = self.out_dims
        cat, lnm, stm, M2 = self.msaved
        dlnm = torch.empty_like(lnm)
        self.red.bwd(lnm, 8 * C, dy, 2 * C, M2, dlnm, 8 * C, accumulate)
        dcat = torch.empty_like(cat)
        self.mnorm.bwd(cat, 8 * C, stm, dlnm, 8 * C, dcat, 8 * C, M2, False, accumulate)
        del dlnm
        dx = torch.empty(N * d * h * w * C, dtype=rt.dtype, device=rt.device)
        L.mmseg_merge_scatter(ptr(dcat), N, d, h, w, C, ptr(dx), C, rt.code, rt.stream)
        del dcat
        for b, st in zip(reversed(self.blocks), reversed(self.saved)):
            dx = b.bwd(dx, st, self.geo, accumulate)
        self.saved, self.msaved = None, None
        return dx


class ResBlockProg:
    """UnetResBlock: conv1 -> IN -> lrelu -> conv2 -> IN, + (conv3 1x1 -> IN | identity), lrelu.  Convs have
    no bias; IN has no affine (MONAI "instance")."""

    def __init__(self, rt: Runtime, blk: nn.Module, flat: FlatParams, cin: int, cout: int, cin_ld: int,
                 first: bool = False):
        self.rt, self.cin, self.cout = rt, cin, cout
        self.cip = cin_ld if first else cpad(cin)
        self.cop = cpad(cout)
        # pad_cols: the a1 / a2 / dh / da buffers own their padded channels (zero-filled by the GEMMs); the
        # input gradient dx of conv1 is a whole buffer too (dcat, or the block's own dx)
        self.c1 = Conv3(rt, blk.conv1.conv, flat, cin_pad=self.cip, need_dgrad=not first, cout_pad=self.cop,
                        pad_cols=True)
        self.c2 = Conv3(rt, blk.conv2.conv, flat, cin_pad=self.cop, cout_pad=self.cop, pad_cols=True)
        self.has3 = hasattr(blk, "conv3")
        self.c3 = Lin(rt, blk.conv3.conv.weight, None, flat, cin_pad=self.cip if first else None,
                      need_dgrad=not first) if self.has3 else None
        self.first = first

    def descs(self):
        d = self.c1.descs() + self.c2.descs()
        return d + (self.c3.descs() if self.has3 else [])

    def setup(self, N, D, H, W):
        rt = self.rt
        z = lambda: Act(torch.zeros(N * D * H * W * self.cop, dtype=rt.dtype, device=rt.device), 0, self.cout,
                        self.cop, N, D, H, W, whole=True)
        self.a1, self.h1, self.a2, self.g, self.da, self.dh = z(), z(), z(), z(), z(), z()
        self.a3 = z() if self.has3 else None
        f = lambda: torch.empty(N * self.cout, dtype=torch.float32, device=rt.device)
        self.m1, self.r1, self.m2, self.r2 = f(), f(), f(), f()
        self.m3, self.r3 = (f(), f()) if self.has3 else (None, None)
        if not self.first:
            self.dres = Act(torch.zeros(N * D * H * W * self.cip, dtype=rt.dtype, device=rt.device), 0, self.cin,
                            self.cip, N, D, H, W) if self.has3 else None
        # the tail's LeakyReLU backward and the norms' partial sums in one pass (mmseg_lrelu_bwd_in_part) above the
        # one-launch small-volume norms; MMSEG_RES_FUSE=0 keeps the separate passes (bitwise the same)
        V = D * H * W
        nch = rt.lib.mmseg_instnorm_part_chunks(V, self.cout) if V > 4096 else 0
        self.res_nch = nch if _res_fuse() else 0
        if self.res_nch:
            p = lambda: torch.empty(N * nch * self.cout * 2, dtype=torch.float32, device=rt.device)
            self.pa, self.pb = p(), (p() if self.has3 else None)

    def _stats(self, a: Act, m, r):
        L = self.rt.lib
        ws = self.rt.ws(L.mmseg_instnorm_ws_floats(a.N, a.V, a.C))
        L.mmseg_instnorm_stats(a.ptr, a.ld, a.N, a.V, a.C, IN_EPS, ptr(m), a.C, ptr(r), ptr(ws), self.rt.code,
                               self.rt.stream)

    def _in_bwd(self, a: Act, m, r, g: Act, dx: Act, part: Optional[torch.Tensor] = None):
        """part: the partial sums mmseg_lrelu_bwd_in_part emitted (finalize + apply only)."""
        self._in_act_bwd(a, m, r, g, dx, 0, part)

    def _in_act_bwd(self, a: Act, m, r, g: Act, dx: Act, act: int, part: Optional[torch.Tensor] = None):
        """The norm's backward with the activation after it (0 none, 2 LeakyReLU) folded in; dx written whole-row."""
        L = self.rt.lib
        ws = self.rt.ws(L.mmseg_instnorm_ws_floats(a.N, a.V, a.C))
        L.mmseg_instnorm_act_bwd(a.ptr, a.ld, ptr(m), ptr(r), g.ptr, g.ld, dx.ptr, dx.ld, a.N, a.D, a.H, a.W, a.C,
                                 dx.wcols if _res_fuse() else a.C, act, SLOPE, ptr(part),
                                 self.res_nch if part is not None else 0, ptr(ws), self.rt.code, self.rt.stream)

    def fwd(self, x: Act, y: Act):
        L, s, code = self.rt.lib, self.rt.stream, self.rt.code
        self.c1.fwd(x, self.a1)
        self._stats(self.a1, self.m1, self.r1)
        L.mmseg_res_apply(self.a1.ptr, self.a1.ld, ptr(self.m1), ptr(self.r1), None, 0, None, None, self.h1.ptr,
                          self.h1.ld, x.N, x.V, self.cout, _wc(self.h1), SLOPE, code, s)
        self.c2.fwd(self.h1, self.a2)
        self._stats(self.a2, self.m2, self.r2)
        if self.has3:
            self.c3.fwd(x.ptr, x.ld, x.N * x.V, self.a3.ptr, self.a3.ld, ncols=_wc(self.a3))
            self._stats(self.a3, self.m3, self.r3)
            L.mmseg_res_apply(self.a2.ptr, self.a2.ld, ptr(self.m2), ptr(self.r2), self.a3.ptr, self.a3.ld,
                              ptr(self.m3), ptr(self.r3), y.ptr, y.ld, x.N, x.V, self.cout, _wc(y), SLOPE, code, s)
        else:
            L.mmseg_res_apply(self.a2.ptr, self.a2.ld, ptr(self.m2), ptr(self.r2), x.ptr, x.ld, None, None, y.ptr,
                              y.ld, x.N, x.V, self.cout, _wc(y), SLOPE, code, s)

    def bwd(self, x: Act, y: Act, dy: Act, dx: Optional[Act], accumulate: bool):
        """dx (if not None) := the input gradient (it must not alias dy)."""
        L, s, code = self.rt.lib, self.rt.stream, self.rt.code
        rows = x.N * x.V
        pa = pb = None
        if self.res_nch:
            a2, a3 = self.a2, self.a3
            pa, pb = self.pa, self.pb
            L.mmseg_lrelu_bwd_in_part(y.ptr, y.ld, dy.ptr, dy.ld, self.g.ptr, self.g.ld, SLOPE, a2.ptr, a2.ld,
                                      ptr(self.m2), ptr(self.r2), ptr(pa), a3.ptr if a3 else None, a3.ld if a3 else 0,
                                      ptr(self.m3), ptr(self.r3), ptr(pb), x.N, x.V, self.cout, _wc(self.g), code, s)
        else:
            L.mmseg_lrelu_bwd(y.ptr, y.ld, dy.ptr, dy.ld, self.g.ptr, self.g.ld, rows, self.cout, _wc(self.g), SLOPE,
                              code, s)
        self._in_bwd(self.a2, self.m2, self.r2, self.g, self.da, pa)
        self.c2.bwd(self.h1, self.da, self.dh, accumulate)
        # h1 = lrelu(IN(a1)): the LeakyReLU's backward inside the norm's passes (h1 > 0 exactly where a1 > mean)
        self._in_act_bwd(self.a1, self.m1, self.r1, self.dh, self.da, 2)
        self.c1.bwd(x, self.da, dx, accumulate)
        if self.has3:
            self._in_bwd(self.a3, self.m3, self.r3, self.g, self.da, pb)
            if dx is not None and self.c3.dgrad_splits(rows, _wc(dx)) == 1 and _res_fuse():
                # dx += d(conv3 branch) from the 1x1 data-gradient GEMM's epilogue (no dres buffer, no add pass)
                self.c3.bwd(x.ptr, x.ld, self.da.ptr, self.da.ld, rows, dx.ptr, dx.ld, accumulate, dx_add=True,
                            dx_cols=_wc(dx))
            else:
                self.c3.bwd(x.ptr, x.ld, self.da.ptr, self.da.ld, rows, self.dres.ptr if dx is not None else None,
                            self.dres.ld if dx is not None else 0, accumulate)
                if dx is not None:
                    _add_act(self.rt, dx, self.dres)
        elif dx is not None:
            _add_act(self.rt, dx, self.g)


def _wc(a: Act) -> int:
    """Channels the pass writing a writes (Act.wcols: whole rows, zeros in the padding), or only the real ones
    (MMSEG_RES_FUSE=0)."""
    return a.wcols if _res_fuse() else a.C


def _add_act(rt: Runtime, dst: Act, src: Act):
    """dst[:, :C] += src[:, :C] over whole rows (both padded to the same ld: the pad channels add finite
    values the zero weights ignore)."""
    if dst.ld != src.ld or dst.off or src.off:
        raise ValueError("residual add: buffers must share the padded layout")
    n = dst.N * dst.V * dst.ld
    rt.lib.mmseg_add(dst.ptr, src.ptr, dst.ptr, n, rt.code, rt.stream)


class UpBlockProg:
    """UnetrUpBlock: ConvTranspose3d(k2 s2, no bias) -> cat([up, skip]) -> UnetResBlock(2C -> C)."""

    def __init__(self, rt: Runtime, blk: nn.Module, flat: FlatParams, cin: int, cout: int):
        self.rt, self.cin, self.cout = rt, cin, cout
        self.up = ConvT2(rt, blk.transp_conv.conv, flat, cout_pad=cpad(cout))
        self.res = ResBlockProg(rt, blk.conv_block, flat, 2 * cout, cout, cpad(2 * cout))

    def descs(self):
        return self.up.descs() + self.res.descs()

    def setup(self, N, D, H, W):
        rt, c, ld = self.rt, self.cout, cpad(2 * self.cout)
        self.cat = Act(torch.zeros(N * D * H * W * ld, dtype=rt.dtype, device=rt.device), 0, 2 * c, ld, N, D, H, W)
        self.dcat = Act(torch.zeros(N * D * H * W * ld, dtype=rt.dtype, device=rt.device), 0, 2 * c, ld, N, D, H, W,
                        whole=True)
        self.res.setup(N, D, H, W)

    def skip(self) -> Act:
        return self.cat.slot(self.cout, self.cout)

    def dskip(self) -> Act:
        return self.dcat.slot(self.cout, self.cout)

    def fwd(self, x: Act, y: Act):
        self.up.fwd(x, self.cat.slot(0, self.cout))
        self.res.fwd(self.cat, y)

    def bwd(self, x: Act, y: Act, dy: Act, dx: Act, accumulate: bool):
        self.res.bwd(self.cat, y, dy, self.dcat, accumulate)
        self.up.bwd(x, self.dcat.slot(0, self.cout), dx, accumulate)


class SwinUNETRProgram:
    """MONAI SwinUNETR.forward / backward (see oracle/swin_oracle.py:swin_unetr_forward)."""

    def __init__(self, rt: Runtime, m: nn.Module, flat: FlatParams):
        net = m.model
        self.rt, self.m, self.net, self.flat = rt, m, net, flat
        fs, self.cin = m.feature_size, m.in_channels
        if self.cin > 8:
            raise ValueError("SwinUNETR engine: at most 8 input channels")
        self.fs = fs
        vit = net.swinViT
        self.embed = Lin(rt, vit.patch_embed.proj.weight, vit.patch_embed.proj.bias, flat,
                         cin_pad=round_up(8 * self.cin, 8), need_dgrad=False)
        self.kp = round_up(8 * self.cin, 8)
        self.stages = [SwinStageProg(rt, getattr(vit, f"layers{i + 1}")[0], flat, fs << i, m.num_heads[i],
                                     m.window_size) for i in range(4)]
        self.pout = [LN(rt, None, fs << i, flat) for i in range(5)]
        self.enc1 = ResBlockProg(rt, net.encoder1.layer, flat, self.cin, fs, 8, first=True)
        self.enc2 = ResBlockProg(rt, net.encoder2.layer, flat, fs, fs, cpad(fs))
        self.enc3 = ResBlockProg(rt, net.encoder3.layer, flat, 2 * fs, 2 * fs, cpad(2 * fs))
        self.enc4 = ResBlockProg(rt, net.encoder4.layer, flat, 4 * fs, 4 * fs, cpad(4 * fs))
        self.enc10 = ResBlockProg(rt, net.encoder10.layer, flat, 16 * fs, 16 * fs, cpad(16 * fs))
        self.dec = [UpBlockProg(rt, getattr(net, f"decoder{k}"), flat, c_in, c_out)
                    for k, c_in, c_out in ((5, 16 * fs, 8 * fs), (4, 8 * fs, 4 * fs), (3, 4 * fs, 2 * fs),
                                           (2, 2 * fs, fs), (1, fs, fs))]
        self.head = Head(rt, net.out.conv.conv, flat)
        self.drop_rate = float(getattr(m, "drop_rate", 0.0))
        self.drop = Drop(rt, self.drop_rate) if self.drop_rate > 0 else None
        self.pos_seed = None
        self.shape = None
        self._packed = None

    def _descs(self):
        d = self.embed.descs()
        for st in self.stages:
            d += st.descs()
        for b in (self.enc1, self.enc2, self.enc3, self.enc4, self.enc10):
            d += b.descs()
        for u in self.dec:
            d += u.descs()
        return d

    def packer(self) -> Packer:
        if self._packed is None:
            self._packed = Packer(self.rt, self._descs())
        return self._packed

    def pack(self):
        """Every packed weight image of the network in two launches (layers.Packer); skipped while a step graph
        with the fused AdamW + pack launch is captured (trainer/step_graph.py)."""
        if getattr(self, "skip_pack", False):
            return
        pk = self.packer()
        v = self.flat.version()
        if pk.fresh != v:
            pk.run()
            pk.fresh = v

    def setup(self, N, D, H, W):
        if self.shape == (N, D, H, W):
            return
        if D % 32 or H % 32 or W % 32:
            raise ValueError(f"SwinUNETR: spatial dims {D}x{H}x{W} must be divisible by 32 (MONAI's own check)")
        self.shape = (N, D, H, W)
        rt, fs = self.rt, self.fs
        g = [(D >> (i + 1), H >> (i + 1), W >> (i + 1)) for i in range(5)]   # token grids of hs[0..4]
        self.g = g
        for i, st in enumerate(self.stages):
            st.setup(N, *g[i])
        z = lambda dims, c: Act(torch.zeros(N * dims[0] * dims[1] * dims[2] * cpad(c), dtype=rt.dtype,
                                            device=rt.device), 0, c, cpad(c), N, *dims, whole=True)
        full = (D, H, W)
        self.xin = Act(torch.zeros(N * D * H * W * 8, dtype=rt.dtype, device=rt.device), 0, self.cin, 8, N, *full)
        # decoder k (5..1) runs at grid of hs[k-2] x2 = g[k-2] for k >= 2 ... decoder1 at full res
        dgrid = [g[3], g[2], g[1], g[0], full]
        for u, dims in zip(self.dec, dgrid):
            u.setup(N, *dims)
        self.enc1.setup(N, *full)
        self.enc2.setup(N, *g[0])
        self.enc3.setup(N, *g[1])
        self.enc4.setup(N, *g[2])
        self.enc10.setup(N, *g[4])
        self.hs = [z(g[0], fs), z(g[1], 2 * fs), z(g[2], 4 * fs), self.dec[0].skip(), z(g[4], 16 * fs)]
        self.dhs = [z(g[0], fs), z(g[1], 2 * fs), z(g[2], 4 * fs), self.dec[0].dskip(), z(g[4], 16 * fs)]
        self.dec4 = z(g[4], 16 * fs)
        self.ddec4 = z(g[4], 16 * fs)
        # decoder outputs: decoder5 -> g[3] (8fs), 4 -> g[2], 3 -> g[1], 2 -> g[0], 1 -> full
        self.dout = [z(dgrid[i], c) for i, c in enumerate((8 * fs, 4 * fs, 2 * fs, fs, fs))]
        self.ddout = [z(dgrid[i], c) for i, c in enumerate((8 * fs, 4 * fs, 2 * fs, fs, fs))]
        self.patches = torch.empty(N * g[0][0] * g[0][1] * g[0][2] * self.kp, dtype=rt.dtype, device=rt.device)

    def forward(self, x: torch.Tensor, training: bool) -> torch.Tensor:
        N, Cx, D, H, W = x.shape
        if Cx != self.cin:
            raise ValueError(f"SwinUNETR: expected {self.cin} input channels, got {Cx}")
        self.setup(N, D, H, W)
        rt, L, s, code, fs = self.rt, self.rt.lib, self.rt.stream, self.rt.code, self.fs
        self.pack()
        g = self.g
        # swinViT
        L.mmseg_patchify(ptr(x), N, Cx, D, H, W, self.kp, ptr(self.patches), code, s)
        M0 = N * g[0][0] * g[0][1] * g[0][2]
        x0 = torch.empty(M0 * fs, dtype=rt.dtype, device=rt.device)
        self.embed.fwd(self.patches, self.kp, M0, x0, fs)
        drop = self.drop if training else None
        self.pos_seed = Drop.seed() if drop is not None else None
        if drop is not None:              # SwinTransformer.pos_drop on patch_embed's NCDHW output
            V0 = g[0][0] * g[0][1] * g[0][2]
            drop(x0, x0, M0, fs, self.pos_seed, V=V0, ncdhw=True)
        xs = [x0]
        h = x0
        for st in self.stages:
            h = st.fwd(h, drop)
            xs.append(h)
        # dropout seeds of this forward by site (the tests regenerate the masks from them)
        self.drop_seeds = {"pos": self.pos_seed} if drop is not None else {}
        if drop is not None:
            for i, st in enumerate(self.stages):
                for j, sv in enumerate(st.saved):
                    self.drop_seeds[f"swinViT.layers{i + 1}.0.blocks.{j}."] = sv["seeds"]
        self.xs = xs
        self.pst = []
        for i in range(5):
            c = fs << i
            rows = N * g[i][0] * g[i][1] * g[i][2]
            hs = self.hs[i]
            self.pst.append(self.pout[i].fwd(xs[i], c, rows, hs.ptr, hs.ld))
        # UNETR
        L.mmseg_pack_input(ptr(x), Cx, 0, Cx, N, D * H * W, self.xin.ptr, code, s)
        self.enc1.fwd(self.xin, self.dec[4].skip())
        self.enc2.fwd(self.hs[0], self.dec[3].skip())
        self.enc3.fwd(self.hs[1], self.dec[2].skip())
        self.enc4.fwd(self.hs[2], self.dec[1].skip())
        self.enc10.fwd(self.hs[4], self.dec4)
        prev = self.dec4
        for u, out in zip(self.dec, self.dout):
            u.fwd(prev, out)
            prev = out
        logits = torch.empty(N, self.head.C, D, H, W, dtype=torch.float32, device=rt.device)
        self.head.fwd(prev, logits, None)
        return logits

    def backward(self, dlogits: torch.Tensor, accumulate: bool):
        rt, L, s, code, fs = self.rt, self.rt.lib, self.rt.stream, self.rt.code, self.fs
        g = self.g
        N = self.shape[0]
        self.head.bwd(self.dout[4], dlogits, self.ddout[4], accumulate)
        ins = [self.dec4] + self.dout[:4]
        dins = [self.ddec4] + self.ddout[:4]
        skip_enc = {4: self.enc1, 3: self.enc2, 2: self.enc3, 1: self.enc4}
        enc_in = {4: self.xin, 3: self.hs[0], 2: self.hs[1], 1: self.hs[2]}
        enc_din = {4: None, 3: self.dhs[0], 2: self.dhs[1], 1: self.dhs[2]}
        for j in range(4, -1, -1):
            u = self.dec[j]
            u.bwd(ins[j], self.dout[j], self.ddout[j], dins[j], accumulate)
            if j in skip_enc:
                skip_enc[j].bwd(enc_in[j], u.skip(), u.dskip(), enc_din[j], accumulate)
        self.enc10.bwd(self.hs[4], self.dec4, self.ddec4, self.dhs[4], accumulate)
        # swinViT: d x_i = proj_out_bwd(d hs_i) + (stage i+1 backward)
        dx = None
        for i in range(4, -1, -1):
            c = fs << i
            rows = N * g[i][0] * g[i][1] * g[i][2]
            if dx is None:
                dx = torch.empty(rows * c, dtype=rt.dtype, device=rt.device)
                add = False
            else:
                add = True
            dh = self.dhs[i]
            self.pout[i].bwd(self.xs[i], c, self.pst[i], dh.ptr, dh.ld, dx, c, rows, add, False)
            if i > 0:
                dx = self.stages[i - 1].bwd(dx, accumulate)
        M0 = N * g[0][0] * g[0][1] * g[0][2]
        if self.pos_seed is not None:
            self.drop(dx, dx, M0, fs, self.pos_seed, V=g[0][0] * g[0][1] * g[0][2], ncdhw=True)
        self.embed.bwd(self.patches, self.kp, dx, fs, M0, None, 0, accumulate)
        self.xs = None
