"""Whole-network programs: UNet3D and DualEncoder forward / backward as fixed
kernel sequences over buffers planned once per input shape.

Memory plan (per level l, spatial S/2^l, F[l] channels, NDHWC):
  cat[l]   [N, V_l, 2F[l]]  decoder input: [:F] = upsampled, [F:] = skip.
           The encoder (UNet) or the fusion kernel (DualEncoder) writes the
           skip straight into its slot and the transposed conv writes the
           upsampled half, so torch.cat (reference unet.py:111) never runs.
  pooled[l], idx[l]         MaxPool3d output + argmax (uint8) feeding level l.
  dcat / dd / dp            backward tensors alias cat / decoder outputs /
                            pooled (their last forward reader has run).
"""
from __future__ import annotations

import contextlib
import ctypes
import os
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn

from .._lib import ptr
from .layers import Block, ConvT2, DySpec, GroupBlock, Head, Packer, Point, act_group_view
from .runtime import Act, FlatParams, Runtime


SMALL_IN_V = 4096   # norm_pool.hip knob_small_v(): at or below it InstanceNorm is one launch (stats + apply)


def _check_dims(D, H, W, levels):
    f = 1 << (levels - 1)
    if D % f or H % f or W % f:
        raise ValueError(
            f"spatial dims {D}x{H}x{W} must be divisible by {f} (the reference's size-mismatch "
            "interpolate branch, unet.py:108-109, is not on the engine path)")


class _Decoder:
    """Shared decoder + head of UNet3D / DualEncoder (reference unet.py:189-196)."""

    def __init__(self, rt: Runtime, up_blocks: nn.ModuleList, out_conv: nn.Conv3d, dropout: float,
                 flat: FlatParams, features: List[int]):
        self.rt, self.F = rt, features
        self.ups = [ConvT2(rt, d.up, flat) for d in up_blocks]
        self.blocks = [Block(rt, d.conv, flat) for d in up_blocks]
        self.head = Head(rt, out_conv, flat)
        self.p = dropout

    def descs(self):
        d = []
        for u in self.ups:
            d += u.descs()
        for b in self.blocks:
            d += b.descs()
        return d

    def setup(self, N, dims):
        rt, F = self.rt, self.F
        self.cat = [rt.act(N, *dims[l], 2 * F[l]) for l in range(len(F) - 1)]
        self.dout = [rt.act(N, *dims[l], F[l]) for l in range(len(F) - 1)]
        # backward: d(cat) as two DENSE tensors over cat's memory (d(upsampled) in its first half, d(skip) in the
        # second), written by the first conv's split data gradient.  Interleaved [voxel][2F], every reader of one
        # half (the transposed conv's backward, the encoders' InstanceNorm backward) fetched full cache lines for
        # half of them: 79 vs 39 us for the 96^3 IN backward partial pass (tools/inbench.py)
        self.dsplit = []
        for l in range(len(F) - 1):
            c = self.cat[l]
            half = c.N * c.V * F[l]
            self.dsplit.append((Act(c.buf, 0, F[l], F[l], c.N, c.D, c.H, c.W),
                                Act(c.buf, half, F[l], F[l], c.N, c.D, c.H, c.W)))
        self.split_bwd = False

    def skip_slot(self, l: int) -> Act:
        return self.cat[l].slot(self.F[l], self.F[l])

    def dskip(self, l: int) -> Act:
        """Gradient of the skip input of decoder level l (valid after bwd)."""
        return self.dsplit[l][1] if self.split_bwd else self.skip_slot(l)

    def fwd(self, bottom: Act, training: bool, loss=None):
        """-> logits; with loss = (labels, spec, class_w): the loss scalar (fused head + loss, no logits)."""
        h = bottom
        nl = len(self.F) - 1
        # the fused head + loss applies the last block's InstanceNorm + ReLU on load, so the training forward
        # never writes that block's output (113 MB at 96^3 B=2)
        self.defer_head = loss is not None and os.environ.get("MMSEG_DEFER_HEAD_NORM", "1") != "0"
        for j in range(nl):
            l = nl - 1 - j
            self.ups[j].fwd(h, self.cat[l].slot(0, self.F[l]))
            self.blocks[j].defer_out = self.defer_head and j == nl - 1
            self.blocks[j].fwd(self.cat[l], self.dout[l])
            h = self.dout[l]
        dscale = None
        if training and self.p > 0:
            keep = torch.empty(h.N, h.C, device=self.rt.device).bernoulli_(1.0 - self.p)
            dscale = keep / (1.0 - self.p)
        if loss is not None:
            labels, spec, cw = loss
            if self.defer_head:
                x2, mu, rs = self.blocks[nl - 1].out_stats()
                return self.head.fwd_loss(x2, labels, spec, cw, dscale, norm=(mu, rs))
            return self.head.fwd_loss(h, labels, spec, cw, dscale)
        # fresh logits every call (caching allocator, no copy): callers may keep them
        logits = torch.empty(h.N, self.head.C, h.D, h.H, h.W, dtype=torch.float32, device=self.rt.device)
        self.head.fwd(h, logits, dscale)
        return logits

    def bwd(self, bottom: Act, dlogits: Optional[torch.Tensor], accumulate: bool,
            gout: Optional[torch.Tensor] = None) -> Act:
        """Returns the gradient of `bottom` (aliases `bottom`'s buffer).  gout (a device scalar) instead of
        dlogits: the fused head + loss backward of a forward that ran with `loss`."""
        nl = len(self.F) - 1
        self.split_bwd = True     # d(cat) as two dense tensors (mmseg_conv_gemm_split)
        dh = self.dout[0]
        hpart = None
        if gout is not None:
            hx = self.blocks[nl - 1].out_stats()[0] if self.defer_head else self.dout[0]
            # the head backward also sums the last block's InstanceNorm-backward partials (no partial pass over
            # its 113 MB x2 + dy at 96^3 B=2)
            nch = self.head.in_chunks(hx)
            if nch:
                size = hx.N * nch * hx.C * 2
                if getattr(self, "_hpart", None) is None or self._hpart.numel() != size:
                    self._hpart = torch.empty(size, dtype=torch.float32, device=self.rt.device)
                hpart = (self._hpart, nch)
            self.head.bwd_loss(hx, gout, dh, accumulate, inpart=hpart[0] if hpart else None)
        else:
            self.head.bwd(self.dout[0], dlogits, dh, accumulate)
        for j in reversed(range(nl)):
            l = nl - 1 - j
            dcat = self.dsplit[l] if self.split_bwd else self.cat[l]                  # aliases cat
            self.blocks[j].bwd(self.cat[l], DySpec(p1=dh, part=hpart if j == nl - 1 else None), dcat, accumulate)
            x_up = bottom if j == 0 else self.dout[l + 1]
            dup = self.dsplit[l][0] if self.split_bwd else self.cat[l].slot(0, self.F[l])
            self.ups[j].bwd(x_up, dup, x_up, accumulate)   # dd aliases x_up
            dh = x_up
        return bottom


class UNetProgram:
    """UNet3D (reference unet.py:116-200) on the HIP engine."""

    def __init__(self, rt: Runtime, m: nn.Module, flat: FlatParams):
        self.rt, self.m, self.flat = rt, m, flat
        self.F = list(m.features)
        self.L = len(self.F)
        self.cin = m.in_channels
        if self.cin > 8:
            raise ValueError("UNet3D engine supports up to 8 input channels")
        self.init = Block(rt, m.init_conv, flat, cin_pad=8, need_dgrad=False)
        self.enc = [Block(rt, e.conv, flat) for e in m.encoders]
        self.dec = _Decoder(rt, m.decoders, m.out_conv, m.dropout_p, flat, self.F)
        self.shape = None

    def packer(self) -> Packer:
        if getattr(self, "_packer", None) is None:
            self._packer = Packer(self.rt, self._all_descs())
        return self._packer

    def pack(self):
        """The weights' operand images from the current fp32 weights -- skipped while a step graph whose fused
        AdamW + pack launch keeps them current is captured (trainer/step_graph.py)."""
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
        _check_dims(D, H, W, self.L)
        self.shape = (N, D, H, W)
        rt, F = self.rt, self.F
        dims = [(D >> l, H >> l, W >> l) for l in range(self.L)]
        self.dims = dims
        self.xin = rt.act(N, *dims[0], 8)
        self.dec.setup(N, dims)
        self.pooled = [None] + [rt.act(N, *dims[l], F[l - 1]) for l in range(1, self.L)]
        # d(pooled): over pooled itself (the weight gradient reads pooled before the data gradient overwrites it)
        self.dpooled = self.pooled
        self.idx = [None] + [torch.empty(N * dims[l][0] * dims[l][1] * dims[l][2] * F[l - 1], dtype=torch.uint8,
                                         device=rt.device) for l in range(1, self.L)]
        self.bottom = rt.act(N, *dims[-1], F[-1])

    def _all_descs(self):
        d = self.init.descs()
        for b in self.enc:
            d += b.descs()
        return d + self.dec.descs()

    def level_out(self, l: int) -> Act:
        return self.dec.skip_slot(l) if l < self.L - 1 else self.bottom

    def forward(self, x: torch.Tensor, training: bool, loss=None) -> torch.Tensor:
        N, Cx, D, H, W = x.shape
        self.setup(N, D, H, W)
        L, s, code = self.rt.lib, self.rt.stream, self.rt.code
        self.pack()
        self.xin_v = _pack_input(self.rt, self.init, x, 0, Cx, self.xin)
        self.init.fwd(self.xin_v, self.level_out(0))
        for l in range(1, self.L):
            prev = self.level_out(l - 1)
            d = self.dims[l - 1]
            L.mmseg_maxpool2_fwd(prev.ptr, prev.ld, self.pooled[l].ptr, self.pooled[l].ld, ptr(self.idx[l]), N, *d,
                                 prev.C, code, s)
            self.enc[l - 1].fwd(self.pooled[l], self.level_out(l))
        return self.dec.fwd(self.bottom, training, loss)

    def loss_ok(self) -> bool:
        return self.dec.head.loss_ok(self.dec.dout[0])

    def backward(self, dlogits: Optional[torch.Tensor], accumulate: bool, gout: Optional[torch.Tensor] = None):
        dbottom = self.dec.bwd(self.bottom, dlogits, accumulate, gout)
        dy = DySpec(p1=dbottom)
        for l in range(self.L - 1, 0, -1):
            self.enc[l - 1].bwd(self.pooled[l], dy, self.dpooled[l], accumulate)   # dp aliases pooled (default)
            dy = DySpec(p1=self.dec.dskip(l - 1), pool_dy=self.dpooled[l], pool_idx=self.idx[l])
        self.init.bwd(self.xin_v, dy, None, accumulate)


class DualEncoderProgram:
    """DualEncoder (reference dual_encoder.py:15-204): one encoder per
    modality, per-level fusion (mean / add / concat+1x1 / CrossModalAttention),
    shared decoder."""

    def __init__(self, rt: Runtime, m: nn.Module, flat: FlatParams):
        self.rt, self.m, self.flat = rt, m, flat
        self.F = list(m.features)
        self.L = len(self.F)
        self.M = m.num_modalities
        if self.M > 4:
            raise ValueError("DualEncoder engine supports up to 4 modalities")
        self.fusion = m.fusion_kind
        self.encs = []
        for e in m.encoders:
            blocks = [Block(rt, e["init_conv"], flat, cin_pad=8, need_dgrad=False)]
            blocks += [Block(rt, b.conv, flat) for b in e["blocks"]]
            self.encs.append(blocks)
        self.proj = [Point(rt, p, flat) for p in m.fusion_proj] if self.fusion == "concat" else None
        self.gates = list(m.fusion_layers) if self.fusion == "attention" else None
        self.dec = _Decoder(rt, m.decoder, m.out_conv, m.dropout_p, flat, self.F)
        self.flat = flat
        self.shape = None
        # modality-grouped small levels (mean / add fusion): each level's M copies of a conv keep their packed
        # weight images at one fixed stride, so one launch can serve all M encoders (layers.ConvGroup)
        self.gblocks = {}
        if self.M > 1 and self.fusion in ("mean", "add"):
            for l in range(1, self.L):
                for attr in ("c1", "c2"):
                    convs = [self.encs[mm][l].__dict__[attr] for mm in range(self.M)]
                    for img in ("wf", "wd"):
                        ts = [c.__dict__[img] for c in convs]
                        if any(t.numel() != ts[0].numel() for t in ts):
                            continue
                        comb = torch.zeros(self.M * ts[0].numel(), dtype=ts[0].dtype, device=ts[0].device)
                        for c, k in zip(convs, range(self.M)):
                            c.__dict__[img] = comb[k * ts[0].numel():(k + 1) * ts[0].numel()]
                self.gblocks[l] = GroupBlock([self.encs[mm][l] for mm in range(self.M)])
        self.l0 = self.L          # first grouped level (setup)

    def _all_descs(self):
        d = []
        for blocks in self.encs:
            for b in blocks:
                d += b.descs()
        if self.proj:
            for p in self.proj:
                d += p.descs()
        return d + self.dec.descs()

    def packer(self) -> Packer:
        if getattr(self, "_packer", None) is None:
            self._packer = Packer(self.rt, self._all_descs())
        return self._packer

    def pack(self):
        """The weights' operand images from the current fp32 weights -- skipped while a step graph whose fused
        AdamW + pack launch keeps them current is captured (trainer/step_graph.py)."""
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
        _check_dims(D, H, W, self.L)
        self.shape = (N, D, H, W)
        rt, F, M = self.rt, self.F, self.M
        dims = [(D >> l, H >> l, W >> l) for l in range(self.L)]
        self.dims = dims
        self.xin = [rt.act(N, *dims[0], 8) for _ in range(M)]
        self.xin_v = list(self.xin)
        self.dec.setup(N, dims)
        # per-modality level outputs
        if self.fusion == "concat":
            self.ycat = [rt.act(N, *dims[l], M * F[l]) for l in range(self.L)]
            self.y = [[self.ycat[l].slot(m * F[l], F[l]) for l in range(self.L)] for m in range(M)]
        else:
            self.y = [[rt.act(N, *dims[l], F[l]) for l in range(self.L)] for _ in range(M)]
        # pooled inputs, their gradients and the argmax codes: one [M x N]-sample tensor per level, the modalities'
        # views of it (a grouped op reads all modalities at once, everything else its own view)
        vol = [d[0] * d[1] * d[2] for d in dims]
        self.pooled_c = [None] + [rt.act(M * N, *dims[l], F[l - 1]) for l in range(1, self.L)]
        self.dpooled_c = self.pooled_c   # (gradients over the pooled tensors, as UNetProgram)
        self.idx_c = [None] + [torch.empty(M * N * vol[l] * F[l - 1], dtype=torch.uint8, device=rt.device)
                               for l in range(1, self.L)]
        self.pooled = [[None] + [act_group_view(self.pooled_c[l], m, N) for l in range(1, self.L)] for m in range(M)]
        self.dpooled = self.pooled
        self.idx = [[None] + [self.idx_c[l][m * N * vol[l] * F[l - 1]:(m + 1) * N * vol[l] * F[l - 1]]
                              for l in range(1, self.L)] for m in range(M)]
        self.bottom = rt.act(N, *dims[-1], F[-1])
        self._setup_groups(N)
        self._setup_outnorm(N)
        if self.fusion == "attention":
            self.pooled_mean = [torch.empty(N, M * F[l], dtype=torch.float32, device=rt.device) for l in range(self.L)]
            self.gate_h = [torch.empty(N, M * F[l] // 4, dtype=torch.float32, device=rt.device) for l in range(self.L)]
            self.gate_w = [torch.empty(N, M, dtype=torch.float32, device=rt.device) for l in range(self.L)]
            self.gate_beta = [torch.empty(N, M * F[l], dtype=torch.float32, device=rt.device) for l in range(self.L)]

    def _setup_groups(self, N: int):
        """Grouped levels: the deepest levels whose M encoder blocks take the grouped kernels (12^3 / 6^3 at a
        96^3 input).  Their pooled inputs, outputs and argmax codes are combined [M x N] tensors; the modality
        views (self.pooled / y / idx [m][l]) keep every other reader unchanged."""
        rt, F, M, dims = self.rt, self.F, self.M, self.dims
        self.l0 = self.L
        self.pooled_g, self.dpooled_g, self.y_g, self.idx_g, self.rep = {}, {}, {}, {}, {}
        if not self.gblocks or self.multistream or os.environ.get("MMSEG_GROUP_SMALL", "1") == "0":
            return
        for l in range(self.L - 1, 0, -1):
            gb = self.gblocks[l]
            gb.setup(N, *dims[l])
            xin = self.pooled_c[l]
            if not gb.ok(xin):
                break
            self.pooled_g[l] = xin
            self.dpooled_g[l] = self.dpooled_c[l]
            self.y_g[l] = rt.act(M * N, *dims[l], F[l])
            self.idx_g[l] = self.idx_c[l]
            for mm in range(M):
                self.y[mm][l] = act_group_view(self.y_g[l], mm, N)
            self.l0 = l

    def _setup_outnorm(self, N: int):
        """Levels above the grouped ones (mean / add fusion): each encoder block's output InstanceNorm backward runs
        for all M modalities as one launch sequence (mmseg_instnorm_relu_bwd_group), reading the fused level's
        gradient once instead of M times.  The blocks' pre-norm outputs x2 and statistics become views of one
        [M x N]-sample tensor per level (self.x2c / self.statsc)."""
        rt, F, M, dims = self.rt, self.F, self.M, self.dims
        self.x2c, self.statsc = {}, {}
        self.group_outnorm = (M > 1 and self.fusion in ("mean", "add") and not self.multistream
                              and os.environ.get("MMSEG_GROUP_SMALL", "1") != "0")   # (one switch for grouping)
        if not self.group_outnorm:
            return
        for l in range(min(self.l0, self.L)):
            C = F[l]
            x2c = rt.act(M * N, *dims[l], C)
            stc = torch.empty(4, M * N * C, dtype=torch.float32, device=rt.device)
            for m in range(M):
                b = self.encs[m][l]
                b.setup(N, *dims[l])
                b.x2 = act_group_view(x2c, m, N)
                b.stats = stc[:, m * N * C:(m + 1) * N * C]
            self.x2c[l], self.statsc[l] = x2c, stc

    def fused_out(self, l: int) -> Act:
        return self.dec.skip_slot(l) if l < self.L - 1 else self.bottom

    def dfused(self, l: int) -> Act:
        """d(fused_l) after the decoder backward."""
        return self.dec.dskip(l) if l < self.L - 1 else self.bottom

    def _fuse_fwd(self, l: int):
        L, s, code = self.rt.lib, self.rt.stream, self.rt.code
        out = self.fused_out(l)
        ys = [self.y[m][l] for m in range(self.M)]
        N, V, C = out.N, out.V, out.C
        if self.fusion == "concat":
            self.proj[l].fwd(self.ycat[l], out)
            return
        srcs = _ptr_array([y.ptr for y in ys])
        lds = _int_array([y.ld for y in ys])
        if self.fusion == "attention":
            g = self.gates[l]
            for m, y in enumerate(ys):
                ws = self.rt.ws(L.mmseg_instnorm_ws_floats(N, V, C))
                L.mmseg_instnorm_stats(y.ptr, y.ld, N, V, C, 0.0, self.pooled_mean[l].data_ptr() + m * C * 4,
                                       self.M * C, None, ptr(ws), code, s)
            lin1, lin2 = g.attention[2], g.attention[4]
            L.mmseg_attn_gate_fwd(ptr(self.pooled_mean[l]), ptr(lin1.weight), ptr(lin1.bias), ptr(lin2.weight),
                                  ptr(lin2.bias), ptr(self.gate_h[l]), ptr(self.gate_w[l]), N, self.M * C,
                                  lin1.weight.shape[0], self.M, s)
            L.mmseg_fuse_fwd(srcs, lds, self.M, 1.0, ptr(self.gate_w[l]), out.ptr, out.ld, N, V, C, code, s)
        else:
            wconst = 1.0 if self.fusion == "add" else 1.0 / self.M
            blks = [self.encs[m][l] for m in range(self.M)]
            if blks[0].defer_out:
                st = [b.out_stats() for b in blks]
                L.mmseg_fuse_norm_fwd(_ptr_array([t[0].ptr for t in st]), _int_array([t[0].ld for t in st]),
                                      _ptr_array([t[1].data_ptr() for t in st]), _ptr_array([t[2].data_ptr() for t in st]),
                                      self.M, wconst, None, out.ptr, out.ld, N, V, C, code, s)
            else:
                L.mmseg_fuse_fwd(srcs, lds, self.M, wconst, None, out.ptr, out.ld, N, V, C, code, s)

    def materialize_features(self):
        """Write the encoder outputs the forward left deferred (return_features reads them)."""
        for m in range(self.M):
            for l in range(self.L):
                if self.encs[m][l].defer_out:
                    self.encs[m][l].materialize_out(self.y[m][l])

    # ------------------------------------------------------- modality streams
    # The M encoders are independent until the per-level fusion (forward) and after the decoder backward
    # (backward, mean / add fusion): encoder m runs on HIP stream m (stream 0 = the caller's), so the small
    # 12^3 / 6^3 kernels of one modality fill the CUs the other one leaves idle.  Each stream has its own
    # scratch arena (Runtime.ws); the streams join before the fusion / at the end of the backward.
    def _streams(self):
        main = torch.cuda.current_stream(self.rt.device)
        if not self.multistream:
            return [main] * self.M
        if getattr(self, "_side", None) is None:
            self._side = [torch.cuda.Stream(self.rt.device) for _ in range(self.M - 1)]
        return [main] + self._side

    @property
    def multistream(self) -> bool:
        # off by default: measured 8.61 vs 8.35 ms per 96^3 DualEncoder step (streams from level 1, 2 or 3
        # alike) -- the small levels' kernels did not overlap enough to pay for the cross-stream joins
        return self.M > 1 and os.environ.get("MMSEG_MODALITY_STREAMS", "0") != "0"

    def _on(self, streams, m):
        if streams[m] is streams[0]:
            return contextlib.nullcontext()
        streams[m].wait_stream(streams[0])
        return torch.cuda.stream(streams[m])

    @property
    def stream_level(self) -> int:
        """First level whose encoder work runs on the modality streams: the 96^3 / 48^3 levels fill the chip
        on their own (run concurrently they only contend for L2 / Infinity Cache), the smaller ones do not."""
        return 2

    def _group_fwd_levels(self):
        """Levels l0 .. L-1 for all modalities at once (the maxpool into l0 ran per modality, into the views)."""
        L, code, s = self.rt.lib, self.rt.code, self.rt.stream
        for l in range(self.l0, self.L):
            if l > self.l0:
                prev = self.y_g[l - 1]
                L.mmseg_maxpool2_fwd(prev.ptr, prev.ld, self.pooled_g[l].ptr, self.pooled_g[l].ld,
                                     ptr(self.idx_g[l]), prev.N, *self.dims[l - 1], prev.C, code, s)
            self.gblocks[l].fwd(self.pooled_g[l], self.y_g[l])

    def _enc_fwd_levels(self, m: int, x: torch.Tensor, lo: int, hi: int, group_from: Optional[int] = None):
        """Levels [lo, hi) of modality m; at level group_from only the maxpool runs (its block is grouped)."""
        L, code, s = self.rt.lib, self.rt.code, self.rt.stream
        N, Cx, D, H, W = x.shape
        blocks = self.encs[m]
        for l in range(lo, hi):
            if l == 0:
                self.xin_v[m] = _pack_input(self.rt, blocks[0], x, m, 1, self.xin[m])
                blocks[0].fwd(self.xin_v[m], self.y[m][0])
                continue
            prev = self.y[m][l - 1]
            pb = blocks[l - 1]
            if pb.defer_out:
                x2, mu, rs = pb.out_stats()
                L.mmseg_maxpool2_norm_fwd(x2.ptr, x2.ld, ptr(mu), ptr(rs), self.pooled[m][l].ptr, self.pooled[m][l].ld,
                                          ptr(self.idx[m][l]), N, *self.dims[l - 1], prev.C, code, s)
            else:
                L.mmseg_maxpool2_fwd(prev.ptr, prev.ld, self.pooled[m][l].ptr, self.pooled[m][l].ld,
                                     ptr(self.idx[m][l]), N, *self.dims[l - 1], prev.C, code, s)
            if l == group_from:
                continue
            blocks[l].fwd(self.pooled[m][l], self.y[m][l])

    def forward(self, x: torch.Tensor, training: bool, loss=None) -> torch.Tensor:
        N, Cx, D, H, W = x.shape
        if Cx != self.M:
            raise ValueError(f"DualEncoder expects {self.M} modalities, got {Cx} channels")
        self.setup(N, D, H, W)
        self.pack()
        # mean / add fusion: an encoder level's output IN + ReLU is applied on load by its maxpool and the fusion
        # kernel (its only readers), so the apply pass never writes y (levels above the one-launch small-IN size)
        defer = self.fusion in ("mean", "add") and os.environ.get("MMSEG_DEFER_ENC_NORM", "1") != "0"
        for m in range(self.M):
            for l in range(self.L):
                d = self.dims[l]
                self.encs[m][l].defer_out = defer and d[0] * d[1] * d[2] > SMALL_IN_V
        streams = self._streams()
        split = min(max(self.stream_level, 0), self.L)
        if self.l0 < self.L:
            # grouped small levels: modality after modality down to the maxpool into level l0, then every op of
            # levels l0 .. L-1 as one launch for all modalities
            for m in range(self.M):
                self._enc_fwd_levels(m, x, 0, self.l0 + 1, group_from=self.l0)
            self._group_fwd_levels()
        else:
            for m in range(self.M):                  # big levels: one stream, modality after modality
                self._enc_fwd_levels(m, x, 0, split)
            for m in range(self.M):                  # small levels: modality m on stream m
                with self._on(streams, m):
                    self._enc_fwd_levels(m, x, split, self.L)
        for m in range(1, self.M):
            if streams[m] is not streams[0]:
                streams[0].wait_stream(streams[m])
        for l in range(self.L):
            self._fuse_fwd(l)
        return self.dec.fwd(self.bottom, training, loss)

    def loss_ok(self) -> bool:
        return self.dec.head.loss_ok(self.dec.dout[0])

    def backward(self, dlogits: Optional[torch.Tensor], accumulate: bool, gout: Optional[torch.Tensor] = None):
        L, s, code = self.rt.lib, self.rt.stream, self.rt.code
        self.dec.bwd(self.bottom, dlogits, accumulate, gout)
        M = self.M
        if self.fusion in ("mean", "add"):
            self._encoders_bwd_streams(accumulate)
            return
        for l in range(self.L - 1, -1, -1):
            dfused = self.dfused(l)
            N, V, C = dfused.N, dfused.V, dfused.C
            base: List[DySpec] = []
            if self.fusion == "concat":
                # 1x1 projection backward: d(ycat) aliases ycat (its wgrad ran first)
                self.proj[l].bwd(self.ycat[l], dfused, self.ycat[l], accumulate)
                base = [DySpec(p1=self.y[m][l]) for m in range(M)]
            elif self.fusion == "attention":
                g = self.gates[l]
                lin1, lin2 = g.attention[2], g.attention[4]
                ys = [self.y[m][l] for m in range(M)]
                ws = self.rt.ws(256 * 4 * N)
                fl = self.flat
                L.mmseg_attn_gate_bwd(_ptr_array([y.ptr for y in ys]), _int_array([y.ld for y in ys]), M,
                                      dfused.ptr, dfused.ld, N, V, C, ptr(self.pooled_mean[l]), ptr(lin1.weight),
                                      ptr(lin2.weight), ptr(self.gate_h[l]), ptr(self.gate_w[l]),
                                      ptr(self.gate_beta[l]), ptr(fl.grad(lin1.weight)), ptr(fl.grad(lin1.bias)),
                                      ptr(fl.grad(lin2.weight)), ptr(fl.grad(lin2.bias)), lin1.weight.shape[0],
                                      ptr(ws), int(accumulate), code, s)
                fl.mark(lin1.weight, lin1.bias, lin2.weight, lin2.bias)
                base = [DySpec(p1=dfused, alpha=self.gate_w[l], alpha_off=m, alpha_stride=M,
                               beta=self.gate_beta[l], beta_off=m * C, beta_stride=M * C) for m in range(M)]
            else:
                sc = 1.0 if self.fusion == "add" else 1.0 / M
                base = [DySpec(p1=dfused, scale1=sc) for _ in range(M)]
            for m in range(M):
                dy = base[m]
                if l < self.L - 1:
                    dy.pool_dy = self.dpooled[m][l + 1]
                    dy.pool_idx = self.idx[m][l + 1]
                blk = self.encs[m][l]
                if l > 0:
                    blk.bwd(self.pooled[m][l], dy, self.dpooled[m][l], accumulate)
                else:
                    blk.bwd(self.xin_v[m], dy, None, accumulate)


    def _encoders_bwd_streams(self, accumulate: bool):
        """Mean / add fusion: every d(fused_l) is final once the decoder backward ran, so modality m's whole
        encoder backward (all levels) is independent of the other modalities' and runs on its own stream."""
        M = self.M
        sc = 1.0 if self.fusion == "add" else 1.0 / M
        streams = self._streams()
        split = min(max(self.stream_level, 0), self.L)

        def levels(m, hi, lo):
            for l in range(hi - 1, lo - 1, -1):
                dy = DySpec(p1=self.dfused(l), scale1=sc)
                if l < self.L - 1:
                    dy.pool_dy = self.dpooled[m][l + 1]
                    dy.pool_idx = self.idx[m][l + 1]
                blk = self.encs[m][l]
                if l > 0:
                    blk.bwd(self.pooled[m][l], dy, self.dpooled[m][l], accumulate)
                else:
                    blk.bwd(self.xin_v[m], dy, None, accumulate)

        if self.l0 < self.L:                          # grouped small levels: all modalities per launch
            for l in range(self.L - 1, self.l0 - 1, -1):
                # every modality group reads the fused gradient's sample n % N (no M-fold copy: -0.03 ms, r04aa)
                p1 = self.dfused(l)
                dy = DySpec(p1=p1, scale1=sc, p1_nmod=p1.N)
                if l < self.L - 1:
                    dy.pool_dy = self.dpooled_g[l + 1]
                    dy.pool_idx = self.idx_g[l + 1]
                self.gblocks[l].bwd(self.pooled_g[l], dy, self.dpooled_g[l], accumulate)   # dp aliases pooled
            if not self.group_outnorm:
                for m in range(M):
                    levels(m, self.l0, 0)
                return
        if self.group_outnorm:
            L, s, code = self.rt.lib, self.rt.stream, self.rt.code
            for l in range(min(self.l0, self.L) - 1, -1, -1):
                # the M output-norm backwards of level l at once, in place over the combined pre-norm outputs
                x2c, stc, p1 = self.x2c[l], self.statsc[l], self.dfused(l)
                NG = x2c.N
                ws = self.rt.ws(L.mmseg_instnorm_ws_floats(NG, x2c.V, x2c.C))
                pdy = self.dpooled_c[l + 1] if l < self.L - 1 else None
                L.mmseg_instnorm_relu_bwd_group(x2c.ptr, x2c.ld, ptr(stc[2]), ptr(stc[3]), p1.ptr, p1.ld, sc, p1.N,
                                                pdy.ptr if pdy is not None else None, pdy.ld if pdy is not None else 0,
                                                ptr(self.idx_c[l + 1]) if pdy is not None else None, x2c.ptr, x2c.ld,
                                                NG, *self.dims[l], x2c.C, ptr(ws), code, s)
                for m in range(M):
                    blk = self.encs[m][l]
                    if l > 0:
                        blk.bwd(self.pooled[m][l], None, self.dpooled[m][l], accumulate, out_done=True)
                    else:
                        blk.bwd(self.xin_v[m], None, None, accumulate, out_done=True)
            return
        for m in range(M):                           # small levels: modality m on stream m
            with self._on(streams, m):
                levels(m, self.L, split)
        for m in range(1, M):
            if streams[m] is not streams[0]:
                streams[0].wait_stream(streams[m])
        for m in range(M):                           # big levels: one stream
            levels(m, split, 0)


def _ptr_array(ptrs):
    return (ctypes.c_void_p * len(ptrs))(*ptrs)


def _int_array(vals):
    return (ctypes.c_int * len(vals))(*vals)


def _pack_input(rt, block, x: torch.Tensor, c0: int, cnt: int, xin: Act) -> Act:
    """Pack channels [c0, c0+cnt) of the NCDHW input for `block`'s first conv.  When that conv takes the stem
    path (stem.hip) the channels are packed without padding into the same buffer (ld = cnt), so the stem's
    halo reads move 2*cnt bytes per voxel instead of 16; otherwise the 8-channel engine layout."""
    N, Ctot, D, H, W = x.shape
    xc = Act(xin.buf, 0, cnt, cnt, xin.N, xin.D, xin.H, xin.W)
    if block.c1._stem(xc, block.Co):
        rt.lib.mmseg_pack_input_compact(ptr(x), Ctot, c0, cnt, N, D * H * W, xc.ptr, rt.code, rt.stream)
        return xc
    rt.lib.mmseg_pack_input(ptr(x), Ctot, c0, cnt, N, D * H * W, xin.ptr, rt.code, rt.stream)
    return xin
