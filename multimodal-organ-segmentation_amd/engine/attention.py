"""Multi-head cross-attention of CrossAttentionFusion (reference
src/models/fusion/attention_fusion.py:77-164) as a fixed sequence of HIP
launches (csrc/attention.hip + the InstanceNorm kernels of norm_pool.hip).

Layout: features are NDHWC [B][V][C] in the engine storage dtype; head h is
the channel slice [h*hd, (h+1)*hd) (the reference's view(B, heads, hd, V),
:141-143), addressed through the batched GEMM's (sample, head) strides.
Every product is `mmseg_bgemm_nt` (C = alpha * A B^T, both operands
K-contiguous); operands that are not are re-laid out by `mmseg_transpose`.

Forward (:129-164)                         Backward
  Qp = q Wq^T + bq  (and Kp, Vp from kv)     dR = IN_bwd(R, dy)            (no ReLU)
  S  = scale * Qp_h Kp_h^T   [B,h,V,V] f32   dO = dR Wo ; gWo = dR^T O ; gbo = colsum dR
  P  = softmax_rows(S)                       dP = dO_h Vp_h^T ; dS = P (dP - rowsum(dP P))
  O_h = P Vp_h                               dVp_h = P^T dO_h ; dQp_h = scale dS Kp_h
  R  = q + O Wo^T + bo                       dKp_h = scale dS^T Qp_h
  y  = InstanceNorm3d(R)                     projections: gW = dY^T X, gb = colsum dY,
                                             dq = dR + dQp Wq, dkv = dKp Wk + dVp Wv
Dropout on attn (:150) is the identity (p = 0, or eval mode).
"""
from __future__ import annotations

from typing import Dict

import torch

from .._lib import ptr
from .runtime import Runtime

F32 = 0
IN_EPS = 1e-5


class CrossAttentionEngine:
    def __init__(self, rt: Runtime, channels: int, heads: int):
        if channels % heads:
            raise ValueError("in_channels must be divisible by num_heads")
        self.rt, self.C, self.h = rt, channels, heads
        self.hd = channels // heads
        if self.hd % 8 or channels % 8:
            raise ValueError("the engine needs head_dim and channels to be multiples of 8")
        self.scale = self.hd ** -0.5

    # -------------------------------------------------------------- helpers
    def _empty(self, *shape, f32=False):
        return torch.empty(*shape, dtype=torch.float32 if f32 else self.rt.dtype, device=self.rt.device)

    def _tr(self, src, s_o, s_i, lds, sdt, dst, d_o, d_i, ldd, ddt, batch, inner, rows, cols):
        self.rt.lib.mmseg_transpose(ptr(src), s_o, s_i, lds, sdt, ptr(dst), d_o, d_i, ldd, ddt, batch, inner, rows,
                                    cols, self.rt.stream)

    def _gemm(self, a, sa, lda, b, sb, ldb, c, sc, ldc, batch, inner, M, N, K, alpha=1.0, bias=None, acc=False,
              c_f32=False):
        self.rt.lib.mmseg_bgemm_nt(ptr(a), sa[0], sa[1], lda, ptr(b), sb[0], sb[1], ldb, ptr(c), sc[0], sc[1], ldc,
                                   ptr(bias), batch, inner, M, N, K, float(alpha), int(acc),
                                   F32 if c_f32 else self.rt.code, self.rt.code, self.rt.stream)

    def _cast(self, w: torch.Tensor) -> torch.Tensor:
        """fp32 weight [Co][Ci] -> storage dtype, same layout (a 1 x n transpose)."""
        out = self._empty(w.numel())
        self._tr(w, 0, 0, w.numel(), F32, out, 0, 0, 1, self.rt.code, 1, 1, 1, w.numel())
        return out

    def _castT(self, w: torch.Tensor) -> torch.Tensor:
        """fp32 weight [Co][Ci] -> storage dtype [Ci][Co]."""
        C = self.C
        out = self._empty(C * C)
        self._tr(w, 0, 0, C, F32, out, 0, 0, C, self.rt.code, 1, 1, C, C)
        return out

    def _from_ncdhw(self, x: torch.Tensor) -> torch.Tensor:
        B, C = x.shape[:2]
        V = x[0, 0].numel()
        out = self._empty(B * V * C)
        self._tr(x, C * V, 0, V, F32, out, V * C, 0, C, self.rt.code, B, 1, C, V)
        return out

    def _to_ncdhw(self, t: torch.Tensor, like: torch.Tensor) -> torch.Tensor:
        B, C = like.shape[:2]
        V = like[0, 0].numel()
        out = torch.empty(like.shape, dtype=torch.float32, device=self.rt.device)
        self._tr(t, V * C, 0, C, self.rt.code, out, C * V, 0, V, F32, B, 1, V, C)
        return out

    def _proj(self, x, w_c, bias, out, M, acc=False):
        C = self.C
        self._gemm(x, (0, 0), C, w_c, (0, 0), C, out, (0, 0), C, 1, 1, M, C, C, bias=bias, acc=acc)

    def _wgrad(self, dy, x, gw: torch.Tensor, gb: torch.Tensor, M: int, ws: Dict):
        """gW[co][ci] (+)= sum_v dY[v][co] X[v][ci]; gb[co] (+)= sum_v dY[v][co]."""
        C, L = self.C, self.rt.lib
        dyt, xt = ws["t1"], ws["t2"]
        self._tr(dy, 0, 0, C, self.rt.code, dyt, 0, 0, M, self.rt.code, 1, 1, M, C)
        self._tr(x, 0, 0, C, self.rt.code, xt, 0, 0, M, self.rt.code, 1, 1, M, C)
        self._gemm(dyt, (0, 0), M, xt, (0, 0), M, gw, (0, 0), C, 1, 1, C, C, M, acc=ws["acc"], c_f32=True)
        part = self.rt.ws(256 * C)
        L.mmseg_colsum(ptr(dy), C, C, M, ptr(part), 256, ptr(gb), int(ws["acc"]), self.rt.code, self.rt.stream)

    # -------------------------------------------------------------- forward
    def forward(self, q: torch.Tensor, kv: torch.Tensor, p: Dict[str, torch.Tensor]):
        """q, kv: NCDHW fp32 [B, C, *spatial]; p: {q_w, q_b, k_w, k_b, v_w, v_b, o_w, o_b} fp32.
        Returns (y NCDHW fp32, saved state for backward)."""
        B, C = q.shape[:2]
        V = q[0, 0].numel()
        h, hd = self.h, self.hd
        if V % 8:
            raise ValueError("the engine needs the voxel count to be a multiple of 8")
        M = B * V
        L, s, code = self.rt.lib, self.rt.stream, self.rt.code
        st = {"shape": (B, V)}
        qf, kvf = self._from_ncdhw(q), self._from_ncdhw(kv)
        R = self._from_ncdhw(q)
        wc = {k: self._cast(p[k + "_w"]) for k in ("q", "k", "v", "o")}
        Qp, Kp, Vp = self._empty(M * C), self._empty(M * C), self._empty(M * C)
        self._proj(qf, wc["q"], p["q_b"], Qp, M)
        self._proj(kvf, wc["k"], p["k_b"], Kp, M)
        self._proj(kvf, wc["v"], p["v_b"], Vp, M)
        S = self._empty(B * h * V * V, f32=True)
        hs = (V * C, hd)                                   # (sample, head) strides of a head slice
        ss = (h * V * V, V * V)
        self._gemm(Qp, hs, C, Kp, hs, C, S, ss, V, B * h, h, V, V, hd, alpha=self.scale, c_f32=True)
        P = self._empty(B * h * V * V)
        L.mmseg_softmax_rows(ptr(S), V, ptr(P), V, B * h * V, V, code, s)
        Vt = self._empty(B * h * hd * V)
        ts = (h * hd * V, hd * V)
        self._tr(Vp, V * C, hd, C, code, Vt, ts[0], ts[1], V, code, B * h, h, V, hd)
        O = self._empty(M * C)
        self._gemm(P, ss, V, Vt, ts, V, O, hs, C, B * h, h, V, hd, V)
        self._proj(O, wc["o"], p["o_b"], R, M, acc=True)   # R = q + out_proj(O)
        mean = torch.empty(B * C, dtype=torch.float32, device=self.rt.device)
        rstd = torch.empty(B * C, dtype=torch.float32, device=self.rt.device)
        ws = self.rt.ws(L.mmseg_instnorm_ws_floats(B, V, C))
        L.mmseg_instnorm_stats(ptr(R), C, B, V, C, IN_EPS, ptr(mean), C, ptr(rstd), ptr(ws), code, s)
        y = self._empty(M * C)
        L.mmseg_instnorm_apply(ptr(R), C, ptr(y), C, B, V, C, ptr(mean), ptr(rstd), 0, code, s)
        st.update(qf=qf, kvf=kvf, Qp=Qp, Kp=Kp, Vp=Vp, P=P, O=O, R=R, mean=mean, rstd=rstd)
        return self._to_ncdhw(y, q), st

    # ------------------------------------------------------------- backward
    def backward(self, dy: torch.Tensor, st: Dict, p: Dict[str, torch.Tensor], grads: Dict[str, torch.Tensor],
                 accumulate: bool):
        """dy: NCDHW fp32.  Writes (accumulate: adds) the parameter gradients into grads[...];
        returns (dq, dkv) NCDHW fp32."""
        B, V = st["shape"]
        C, h, hd = self.C, self.h, self.hd
        M = B * V
        L, s, code = self.rt.lib, self.rt.stream, self.rt.code
        dyf = self._from_ncdhw(dy)
        dR = self._empty(M * C)
        ws = self.rt.ws(L.mmseg_instnorm_ws_floats(B, V, C))
        # InstanceNorm3d backward without ReLU (p1 = dy); spatial dims only matter for the pooled gather
        L.mmseg_instnorm_bwd(ptr(st["R"]), C, ptr(st["mean"]), ptr(st["rstd"]), ptr(dyf), C, 1.0, None, 0, None, 0,
                             None, 0, None, ptr(dR), C, B, 1, 1, V, C, 0, ptr(ws), code, s)
        tws = {"t1": self._empty(M * C), "t2": self._empty(M * C), "acc": accumulate}
        wT = {k: self._castT(p[k + "_w"]) for k in ("q", "k", "v", "o")}
        # out_proj
        self._wgrad(dR, st["O"], grads["o_w"], grads["o_b"], M, tws)
        dO = self._empty(M * C)
        self._proj(dR, wT["o"], None, dO, M)
        # attention
        hs, ss = (V * C, hd), (h * V * V, V * V)
        ts = (h * hd * V, hd * V)
        dP = self._empty(B * h * V * V, f32=True)
        self._gemm(dO, hs, C, st["Vp"], hs, C, dP, ss, V, B * h, h, V, V, hd, c_f32=True)
        dS = self._empty(B * h * V * V)
        L.mmseg_softmax_bwd_rows(ptr(st["P"]), V, ptr(dP), V, ptr(dS), V, B * h * V, V, code, s)
        XT = self._empty(B * h * V * V)                    # P^T, then dS^T
        HT = self._empty(B * h * hd * V)                   # per-head [hd][V] operand
        dQp, dKp, dVp = self._empty(M * C), self._empty(M * C), self._empty(M * C)
        # dV_h = P^T dO_h
        self._tr(st["P"], ss[0], ss[1], V, code, XT, ss[0], ss[1], V, code, B * h, h, V, V)
        self._tr(dO, V * C, hd, C, code, HT, ts[0], ts[1], V, code, B * h, h, V, hd)
        self._gemm(XT, ss, V, HT, ts, V, dVp, hs, C, B * h, h, V, hd, V)
        # dQ_h = scale dS K_h
        self._tr(st["Kp"], V * C, hd, C, code, HT, ts[0], ts[1], V, code, B * h, h, V, hd)
        self._gemm(dS, ss, V, HT, ts, V, dQp, hs, C, B * h, h, V, hd, V, alpha=self.scale)
        # dK_h = scale dS^T Q_h
        self._tr(dS, ss[0], ss[1], V, code, XT, ss[0], ss[1], V, code, B * h, h, V, V)
        self._tr(st["Qp"], V * C, hd, C, code, HT, ts[0], ts[1], V, code, B * h, h, V, hd)
        self._gemm(XT, ss, V, HT, ts, V, dKp, hs, C, B * h, h, V, hd, V, alpha=self.scale)
        # projections
        self._wgrad(dQp, st["qf"], grads["q_w"], grads["q_b"], M, tws)
        self._wgrad(dKp, st["kvf"], grads["k_w"], grads["k_b"], M, tws)
        self._wgrad(dVp, st["kvf"], grads["v_w"], grads["v_b"], M, tws)
        self._proj(dQp, wT["q"], None, dR, M, acc=True)     # dq = dR (residual) + dQp Wq
        dkv = self._empty(M * C)
        self._proj(dKp, wT["k"], None, dkv, M)
        self._proj(dVp, wT["v"], None, dkv, M, acc=True)
        return self._to_ncdhw(dR, dy), self._to_ncdhw(dkv, dy)


class FusionHeadEngine:
    """BidirectionalCrossAttention's head (reference attention_fusion.py:196-200, 214):
    y = ReLU(InstanceNorm3d(Conv3d(2C -> C, k=1)(cat([a, b], dim=1)))).  The concatenation is one NDHWC
    [V][2C] buffer both inputs are transposed into (torch.cat never runs); the 1x1 conv and its gradients are
    mmseg_bgemm_nt products, the norm the ReLU-fused InstanceNorm kernels."""

    def __init__(self, rt: Runtime, channels: int):
        self.rt, self.C = rt, channels

    def _empty(self, n, f32=False):
        return torch.empty(n, dtype=torch.float32 if f32 else self.rt.dtype, device=self.rt.device)

    def _tr(self, *a):
        self.rt.lib.mmseg_transpose(*a, self.rt.stream)

    def _gemm(self, a, lda, b, ldb, c, ldc, M, N, K, bias=None, acc=False, c_f32=False):
        self.rt.lib.mmseg_bgemm_nt(ptr(a), 0, 0, lda, ptr(b), 0, 0, ldb, ptr(c), 0, 0, ldc, ptr(bias), 1, 1, M, N, K,
                                   1.0, int(acc), F32 if c_f32 else self.rt.code, self.rt.code, self.rt.stream)

    def forward(self, a: torch.Tensor, b: torch.Tensor, w: torch.Tensor, bias: torch.Tensor):
        B, C = a.shape[:2]
        V = a[0, 0].numel()
        M, L, s, code = B * V, self.rt.lib, self.rt.stream, self.rt.code
        X = self._empty(M * 2 * C)
        for i, t in enumerate((a, b)):     # NCDHW fp32 -> channel slot i of the [V][2C] concat buffer
            self._tr(ptr(t), C * V, 0, V, F32, ptr(X) + i * C * X.element_size(), V * 2 * C, 0, 2 * C, code, B, 1, C,
                     V)
        wc = self._empty(C * 2 * C)
        self._tr(ptr(w), 0, 0, w.numel(), F32, ptr(wc), 0, 0, 1, code, 1, 1, 1, w.numel())
        Z = self._empty(M * C)
        self._gemm(X, 2 * C, wc, 2 * C, Z, C, M, C, 2 * C, bias=bias)
        mean = torch.empty(B * C, dtype=torch.float32, device=self.rt.device)
        rstd = torch.empty(B * C, dtype=torch.float32, device=self.rt.device)
        ws = self.rt.ws(L.mmseg_instnorm_ws_floats(B, V, C))
        L.mmseg_instnorm_stats(ptr(Z), C, B, V, C, IN_EPS, ptr(mean), C, ptr(rstd), ptr(ws), code, s)
        y = self._empty(M * C)
        L.mmseg_instnorm_apply(ptr(Z), C, ptr(y), C, B, V, C, ptr(mean), ptr(rstd), 1, code, s)
        out = torch.empty(a.shape, dtype=torch.float32, device=self.rt.device)
        self._tr(ptr(y), V * C, 0, C, code, ptr(out), C * V, 0, V, F32, B, 1, V, C)
        return out, {"shape": (B, V), "X": X, "Z": Z, "mean": mean, "rstd": rstd}

    def backward(self, dy: torch.Tensor, st, w: torch.Tensor, gw: torch.Tensor, gb: torch.Tensor):
        B, V = st["shape"]
        C, M, L, s, code = self.C, B * V, self.rt.lib, self.rt.stream, self.rt.code
        dyf = self._empty(M * C)
        self._tr(ptr(dy), C * V, 0, V, F32, ptr(dyf), V * C, 0, C, code, B, 1, C, V)
        dZ = self._empty(M * C)
        ws = self.rt.ws(L.mmseg_instnorm_ws_floats(B, V, C))
        L.mmseg_instnorm_bwd(ptr(st["Z"]), C, ptr(st["mean"]), ptr(st["rstd"]), ptr(dyf), C, 1.0, None, 0, None, 0,
                             None, 0, None, ptr(dZ), C, B, 1, 1, V, C, 1, ptr(ws), code, s)
        dZt, Xt = self._empty(C * M), self._empty(2 * C * M)
        self._tr(ptr(dZ), 0, 0, C, code, ptr(dZt), 0, 0, M, code, 1, 1, M, C)
        self._tr(ptr(st["X"]), 0, 0, 2 * C, code, ptr(Xt), 0, 0, M, code, 1, 1, M, 2 * C)
        self._gemm(dZt, M, Xt, M, gw, 2 * C, C, 2 * C, M, c_f32=True)          # gW[co][ci] = sum_v dZ X
        part = self.rt.ws(256 * C)
        L.mmseg_colsum(ptr(dZ), C, C, M, ptr(part), 256, ptr(gb), 0, code, s)
        wt = self._empty(2 * C * C)
        self._tr(ptr(w), 0, 0, 2 * C, F32, ptr(wt), 0, 0, C, code, 1, 1, C, 2 * C)   # W^T [2C][C]
        dX = self._empty(M * 2 * C)
        self._gemm(dZ, C, wt, C, dX, 2 * C, M, 2 * C, C)
        outs = []
        for i in range(2):
            o = torch.empty(B, C, *dy.shape[2:], dtype=torch.float32, device=self.rt.device)
            self._tr(ptr(dX) + i * C * dX.element_size(), V * 2 * C, 0, 2 * C, code, ptr(o), C * V, 0, V, F32, B, 1,
                     V, C)
            outs.append(o)
        return outs


class WindowAttentionEngine:
    """MONAI SwinUNETR WindowAttention (window multi-head self-attention with relative-position bias and the
    shifted-window mask) on the engine: x [B windows, N tokens, C] -> [B, N, C].  The qkv / proj linears, QK^T,
    P.V and every gradient product are mmseg_bgemm_nt (MFMA); the bias gather, the biased softmax and the
    bias-table gradient are csrc/attention.hip kernels.  head_dim = C / heads must be a multiple of 8 (16 in
    SwinUNETR at every stage).  N (343 for a 7^3 window) need not be a multiple of 8: every [*][N] operand
    is stored with its rows padded to ldn = round_up(N, 8) and the padding zeroed, which is what the GEMM's
    K-tail contract asks for (the same for the B*N token dimension of the weight-gradient products)."""

    def __init__(self, rt: Runtime, dim: int, heads: int):
        if dim % heads or (dim // heads) % 8:
            raise ValueError("WindowAttention engine: dim / num_heads must be a multiple of 8")
        self.rt, self.C, self.h, self.hd = rt, dim, heads, dim // heads
        self.scale = self.hd ** -0.5

    def _empty(self, n, f32=False, zero=False):
        f = torch.zeros if zero else torch.empty
        return f(int(n), dtype=torch.float32 if f32 else self.rt.dtype, device=self.rt.device)

    def _tr(self, src, s_o, s_i, lds, sdt, dst, d_o, d_i, ldd, ddt, batch, inner, rows, cols):
        self.rt.lib.mmseg_transpose(ptr(src), s_o, s_i, lds, sdt, ptr(dst), d_o, d_i, ldd, ddt, batch, inner, rows,
                                    cols, self.rt.stream)

    def _gemm(self, a, sa, lda, b, sb, ldb, c, sc, ldc, batch, inner, M, N, K, alpha=1.0, bias=None, acc=False,
              c_f32=False):
        self.rt.lib.mmseg_bgemm_nt(ptr(a), sa[0], sa[1], lda, ptr(b), sb[0], sb[1], ldb, ptr(c), sc[0], sc[1], ldc,
                                   ptr(bias), batch, inner, M, N, K, float(alpha), int(acc),
                                   F32 if c_f32 else self.rt.code, self.rt.code, self.rt.stream)

    def _cast(self, t: torch.Tensor) -> torch.Tensor:
        if self.rt.code == F32:
            return t.contiguous().reshape(-1)
        out = self._empty(t.numel())
        self._tr(t, 0, 0, t.numel(), F32, out, 0, 0, 1, self.rt.code, 1, 1, 1, t.numel())
        return out

    def _castT(self, w: torch.Tensor) -> torch.Tensor:
        """fp32 [R][Cc] -> storage dtype [Cc][R]."""
        R, Cc = w.shape
        out = self._empty(R * Cc)
        self._tr(w, 0, 0, Cc, F32, out, 0, 0, R, self.rt.code, 1, 1, R, Cc)
        return out

    def _to_f32(self, t: torch.Tensor, shape) -> torch.Tensor:
        if self.rt.code == F32:
            return t.view(shape)
        out = torch.empty(shape, dtype=torch.float32, device=self.rt.device)
        self._tr(t, 0, 0, t.numel(), self.rt.code, out, 0, 0, 1, F32, 1, 1, 1, t.numel())
        return out

    def _colsum(self, y, ch, M, out, acc):
        part = self.rt.ws(256 * ch)
        self.rt.lib.mmseg_colsum(ptr(y), ch, ch, M, ptr(part), 256, ptr(out), int(acc), self.rt.code, self.rt.stream)

    def _wgrad(self, dy, ch_out, x, ch_in, M, gw, acc):
        """gW[co][ci] (+)= sum_t dY[t][co] X[t][ci] over the M tokens (token rows padded to ldm, zeroed)."""
        code = self.rt.code
        ldm = (M + 7) // 8 * 8
        t1, t2 = self._empty(ch_out * ldm, zero=True), self._empty(ch_in * ldm, zero=True)
        self._tr(dy, 0, 0, ch_out, code, t1, 0, 0, ldm, code, 1, 1, M, ch_out)
        self._tr(x, 0, 0, ch_in, code, t2, 0, 0, ldm, code, 1, 1, M, ch_in)
        self._gemm(t1, (0, 0), ldm, t2, (0, 0), ldm, gw, (0, 0), ch_in, 1, 1, ch_out, ch_in, M, acc=acc, c_f32=True)

    def core_fwd(self, qkv: torch.Tensor, B: int, N: int, mask, table: torch.Tensor, index: torch.Tensor):
        """Attention core on a qkv buffer [B*N][3C] (storage dtype): softmax(scale q k^T + bias (+ mask)) v
        -> (O [B*N][C], P [B][h][N][ldn]).  table [T][heads] fp32, index int32 [N*N] (device)."""
        C, h, hd = self.C, self.h, self.hd
        M = B * N
        ldn = (N + 7) // 8 * 8
        L, s, code = self.rt.lib, self.rt.stream, self.rt.code
        qs = (N * 3 * C, hd)                        # head-slice strides inside qkv
        ss = (h * N * ldn, N * ldn)                 # [B][h][N][ldn] score-shaped buffers
        S = self._empty(B * h * N * ldn, f32=True)
        self._gemm(qkv, qs, 3 * C, qkv[C:], qs, 3 * C, S, ss, ldn, B * h, h, N, N, hd, alpha=self.scale, c_f32=True)
        bias = self._empty(h * N * N, f32=True)
        L.mmseg_relpos_bias(ptr(table), ptr(index), h, N, ptr(bias), s)
        P = self._empty(B * h * N * ldn)
        nw = mask.shape[0] if mask is not None else 0
        L.mmseg_softmax_bias_rows(ptr(S), ldn, ptr(bias), ptr(mask), nw, h, ptr(P), ldn, B * h * N, N, code, s)
        del S
        ts = (h * hd * ldn, hd * ldn)               # [B][h][hd][ldn] per-head transposed operands
        Vt = self._empty(B * h * hd * ldn, zero=True)
        self._tr(qkv[2 * C:], qs[0], qs[1], 3 * C, code, Vt, ts[0], ts[1], ldn, code, B * h, h, N, hd)
        O = self._empty(M * C)
        hs = (N * C, hd)
        self._gemm(P, ss, ldn, Vt, ts, ldn, O, hs, C, B * h, h, N, hd, N)
        return O, P

    def core_bwd(self, dO: torch.Tensor, qkv: torch.Tensor, P: torch.Tensor, B: int, N: int, gtable: torch.Tensor,
                 csr, accumulate: bool) -> torch.Tensor:
        """Backward of core_fwd: dqkv [B*N][3C] (storage dtype); the bias-table gradient (+)= into gtable."""
        C, h, hd = self.C, self.h, self.hd
        M = B * N
        ldn = (N + 7) // 8 * 8
        L, s, code = self.rt.lib, self.rt.stream, self.rt.code
        qs, ss, hs = (N * 3 * C, hd), (h * N * ldn, N * ldn), (N * C, hd)
        ts = (h * hd * ldn, hd * ldn)
        dP = self._empty(B * h * N * ldn, f32=True)
        self._gemm(dO, hs, C, qkv[2 * C:], qs, 3 * C, dP, ss, ldn, B * h, h, N, N, hd, c_f32=True)
        dS = self._empty(B * h * N * ldn)
        L.mmseg_softmax_bwd_rows(ptr(P), ldn, ptr(dP), ldn, ptr(dS), ldn, B * h * N, N, code, s)
        del dP
        dB = self._empty(h * N * N, f32=True)
        offs, pairs, T = csr
        L.mmseg_relpos_table_grad(ptr(dS), ldn, B, h, N, ptr(dB), ptr(offs), ptr(pairs), T, ptr(gtable),
                                  int(accumulate), code, s)
        dqkv = self._empty(M * 3 * C)
        XT = self._empty(B * h * N * ldn, zero=True)
        HT = self._empty(B * h * hd * ldn, zero=True)
        # dQ_h = scale dS K_h
        self._tr(qkv[C:], qs[0], qs[1], 3 * C, code, HT, ts[0], ts[1], ldn, code, B * h, h, N, hd)
        self._gemm(dS, ss, ldn, HT, ts, ldn, dqkv, qs, 3 * C, B * h, h, N, hd, N, alpha=self.scale)
        # dK_h = scale dS^T Q_h
        self._tr(dS, ss[0], ss[1], ldn, code, XT, ss[0], ss[1], ldn, code, B * h, h, N, N)
        self._tr(qkv, qs[0], qs[1], 3 * C, code, HT, ts[0], ts[1], ldn, code, B * h, h, N, hd)
        self._gemm(XT, ss, ldn, HT, ts, ldn, dqkv[C:], qs, 3 * C, B * h, h, N, hd, N, alpha=self.scale)
        # dV_h = P^T dO_h
        self._tr(P, ss[0], ss[1], ldn, code, XT, ss[0], ss[1], ldn, code, B * h, h, N, N)
        self._tr(dO, hs[0], hs[1], C, code, HT, ts[0], ts[1], ldn, code, B * h, h, N, hd)
        self._gemm(XT, ss, ldn, HT, ts, ldn, dqkv[2 * C:], qs, 3 * C, B * h, h, N, hd, N)
        return dqkv

    def forward(self, x: torch.Tensor, mask, p, index: torch.Tensor):
        """x [B, N, C] fp32; mask [nw, N, N] fp32 or None; p: qkv_w [3C][C], qkv_b [3C] | None, proj_w [C][C],
        proj_b [C], table [T][heads]; index int32 [N*N] (device)."""
        B, N, C = x.shape
        M = B * N
        xf = self._cast(x)
        qkv = self._empty(M * 3 * C)
        self._gemm(xf, (0, 0), C, self._cast(p["qkv_w"]), (0, 0), C, qkv, (0, 0), 3 * C, 1, 1, M, 3 * C, C,
                   bias=p.get("qkv_b"))
        O, P = self.core_fwd(qkv, B, N, mask, p["table"], index)
        y = self._empty(M * C)
        self._gemm(O, (0, 0), C, self._cast(p["proj_w"]), (0, 0), C, y, (0, 0), C, 1, 1, M, C, C, bias=p["proj_b"])
        return self._to_f32(y, (B, N, C)), {"shape": (B, N), "xf": xf, "qkv": qkv, "P": P, "O": O}

    def backward(self, dy: torch.Tensor, st, p, grads, csr, accumulate: bool = False):
        B, N = st["shape"]
        C = self.C
        M = B * N
        qkv, P, O = st["qkv"], st["P"], st["O"]
        dyf = self._cast(dy)
        # proj
        self._wgrad(dyf, C, O, C, M, grads["proj_w"], accumulate)
        self._colsum(dyf, C, M, grads["proj_b"], accumulate)
        dO = self._empty(M * C)
        self._gemm(dyf, (0, 0), C, self._castT(p["proj_w"]), (0, 0), C, dO, (0, 0), C, 1, 1, M, C, C)
        dqkv = self.core_bwd(dO, qkv, P, B, N, grads["table"], csr, accumulate)
        # qkv linear
        self._wgrad(dqkv, 3 * C, st["xf"], C, M, grads["qkv_w"], accumulate)
        if "qkv_b" in grads:
            self._colsum(dqkv, 3 * C, M, grads["qkv_b"], accumulate)
        dx = self._empty(M * C)
        self._gemm(dqkv, (0, 0), 3 * C, self._castT(p["qkv_w"]), (0, 0), 3 * C, dx, (0, 0), C, 1, 1, M, C, 3 * C)
        return self._to_f32(dx, (B, N, C))
