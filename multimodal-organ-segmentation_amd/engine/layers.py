"""Engine layers: each binds an nn.Module parameter container (so state-dict
names, init and checkpoints stay the reference's) to the HIP kernels.

  Conv3      nn.Conv3d(k=3, pad=1)          reference unet.py:26-27
  ConvT2     nn.ConvTranspose3d(k=2, s=2)   reference unet.py:95
  Point      nn.Conv3d(k=1) fusion proj     reference dual_encoder.py:75
  Block      ConvBlock3D = (Conv3 + InstanceNorm3d + ReLU) x 2   unet.py:12-60
  Head       Dropout3d + out_conv 1x1       unet.py:162-163 / dual_encoder.py:83-84

Forward/backward are explicit kernel sequences.  Backward buffers alias
forward buffers whose last reader has already run (weight-gradient GEMMs are
always issued before the data-gradient GEMM that overwrites their input),
so a training step needs no activation memory beyond the forward's.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import List, Optional, Tuple

import torch
import torch.nn as nn

from .._lib import ptr
from .profiler import TIMER
from .runtime import Act, FlatParams, Runtime, pow2_shift, round_up

MODE_CONV3, MODE_POINT, MODE_CONVT_FWD, MODE_CONVT_DGRAD = 0, 1, 2, 3
IN_EPS = 1e-5
TARGET_BLOCKS = 1024


def _own_part(obj, rt: Runtime, nfloats: int) -> torch.Tensor:
    """A split-partial buffer of obj's own (its reduce is queued: Runtime.defer_wred / Runtime.own_part)."""
    return rt.own_part(obj, nfloats)


def _gemm_name(rt: Runtime, ncols: int, mode: str):
    """Timer family = the kernel the library actually launched (same name as in rocprofv3 traces)."""
    return lambda: f"{rt.lib.mmseg_last_kernel().decode()}[{'bf16' if rt.code else 'f32'}]"


def _io_bytes(rt: Runtime, vox: int, cin: int, cout: int, wcount: int, wbytes: int = 2) -> float:
    """Compulsory HBM bytes of one conv launch: read `cin` channels and write `cout` channels of `vox`
    voxels at the storage width, plus the weights (`wcount` values of `wbytes`)."""
    es = rt.dtype.itemsize
    return float(vox * (cin + cout) * es + wcount * wbytes)


def _zcols(a: Act, ncols: int) -> int:
    """Whole-row extent for a GEMM writing ncols columns of a (mmseg_conv_gemm_zw): a's Act.wcols when it reaches past
    ncols, else 0 (no zero columns)."""
    w = a.wcols
    return w if w > ncols and w - ncols <= 48 else 0


def _col_tile(n: int) -> int:
    return round_up(n, 64 if n >= 64 else 32)


def _gemm_ksplit(M: int, ncols: int, KG: int) -> int:
    tiles = -(-M // 128) * -(-ncols // (64 if ncols >= 64 else 32))
    if tiles >= 512 or KG < 32:
        return 1
    return max(1, min(-(-512 // tiles), KG // 16))


class Packer:
    """Weight packing of a whole program per step: every 3^3 conv's two operand images in ONE launch
    (mmseg_pack_conv3_batched: one coalesced read of the fp32 weights), the transposed / 1x1 / token-linear
    images in one more (mmseg_pack_weights_batched)."""

    def __init__(self, rt: Runtime, descs):
        import struct
        self.rt = rt
        self.descs = list(descs)
        # FlatParams.version() the images were last written for (by run() or by the fused AdamW + pack launch);
        # None: unknown -- the next pack writes them
        self.fresh = None
        self._adam = None
        self.per_layer = []
        self.table = self.gtable = None
        if self.per_layer:
            return
        nbytes = rt.lib.mmseg_pack3_desc_bytes()
        blob, begin, n = bytearray(), 0, 0
        dgrad = {d[0]: d for d in descs if d[2] in (1, 6)}
        rest = []
        for d in descs:
            w, dst, mode, Co, Ci, Cip, KG, KGp, Cpad = d
            if mode in (1, 6):
                continue
            if mode != 0:
                rest.append(d)
                continue
            dd = dgrad.get(w)
            cop = dd[5] if dd is not None and dd[2] == 6 else 0
            rec = struct.pack("<QQQ8i", w, dst, dd[1] if dd else 0, Co, Ci, Cip, Cpad, dd[8] if dd else 0, begin, cop,
                              0)
            assert len(rec) == nbytes, (len(rec), nbytes)
            blob += rec
            begin += (Co // 8) * (-(-Ci // 32))
            n += 1
        self.n, self.nblocks = n, begin
        if n:
            self.table = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(rt.device)
        if rest:
            gblob, total = bytearray(), 0
            for (w, dst, mode, Co, Ci, Cip, KG, KGp, Cpad) in rest:
                gblob += struct.pack("<QQ8iq", w, dst, mode, Co, Ci, Cip, KG, KGp, Cpad, 0, total)
                total += KGp * Cpad * 8
            assert len(gblob) == len(rest) * rt.lib.mmseg_pack_desc_bytes()
            self.gtable = torch.frombuffer(gblob, dtype=torch.uint8).to(rt.device)
            self.gn, self.gtotal = len(rest), total

    AP_KT, AP_RANGE = 512, 4096   # conv_gemm.hip: kind-1 tile columns, kind-2 elements per block

    def adam(self, flat) -> Optional[Tuple[torch.Tensor, int, int]]:
        """adam_table(flat), built once per arena."""
        key = (id(flat), flat.flat.data_ptr(), flat.numel)
        if self._adam is None or self._adam[0] != key:
            self._adam = (key, self.adam_table(flat))
        return self._adam[1]

    def adam_table(self, flat) -> Optional[Tuple[torch.Tensor, int, int]]:
        """(device table, descriptors, blocks) of the fused AdamW + pack (mmseg_adamw_pack_dev) over `flat`'s arena:
        every packed weight as tiles that also write its operand images (3^3 convs: kind 0, pack_conv3_batched's
        tiles; 1x1 / token-linear and transposed convs: kind 1), every other arena element in a plain range (kind
        2), each element exactly once.  None when some weight's images do not fit those kinds (the captured step
        then keeps the pack in its forward)."""
        import struct
        if self.per_layer or not self.descs:
            return None
        base, numel = flat.flat.data_ptr(), flat.numel
        groups = {}
        for d in self.descs:
            g = groups.setdefault(d[0], {})
            if d[2] in g and g[d[2]] != d:
                return None          # one weight, two different images of one mode
            g[d[2]] = d
        recs = []
        for w, bym in groups.items():
            modes = sorted(bym)
            if (w - base) % 4:
                return None
            off = (w - base) // 4
            if modes in ([0], [0, 1], [0, 6]):
                f, dd = bym[0], bym.get(1) or bym.get(6)
                Co, Ci, Cip, Cpad = f[3], f[4], f[5], f[8]
                if Co % 8:
                    return None
                rec = (0, off, Co * Ci * 27, (Co // 8) * -(-Ci // 32), f[1], dd[1] if dd else 0, 0, 0, 0, -1, Co, Ci,
                       Cip, Cpad, dd[8] if dd else 0, dd[5] if dd is not None and dd[2] == 6 else 0)
            elif modes in ([2], [2, 3]):
                f, dd = bym[2], bym.get(3)
                Co, Ci = f[3], f[4]
                if Co % 8:
                    return None
                rec = (1, off, Co * Ci, (Co // 8) * -(-Ci // self.AP_KT), f[1], dd[1] if dd else 0, Co, Ci, 2,
                       3 if dd else -1, Co, Ci, 0, f[8], dd[8] if dd else 0, 0)
            elif modes in ([4], [4, 5], [4, 7]):
                f, dd = bym[4], bym.get(5) or bym.get(7)
                Co, Ci = f[3], f[4]
                if Co % 8 or Ci % 8:
                    return None
                rec = (1, off, Ci * Co * 8, (Ci // 8) * -(-(Co * 8) // self.AP_KT), f[1], dd[1] if dd else 0, Ci,
                       Co * 8, 4, dd[2] if dd else -1, Co, Ci, 0, f[8], dd[8] if dd else 0,
                       dd[5] if dd is not None and dd[2] == 7 else 0)
            else:
                return None
            if off < 0 or off + rec[2] > numel:
                return None
            recs.append(rec)
        recs.sort(key=lambda r: r[1])
        full, pos = [], 0
        for r in recs:
            if r[1] < pos:
                return None          # overlapping weights
            if r[1] > pos:
                n = r[1] - pos
                full.append((2, pos, n, -(-n // self.AP_RANGE), 0, 0, 0, n, 0, -1, 0, 0, 0, 0, 0, 0))
            full.append(r)
            pos = r[1] + r[2]
        if pos < numel:
            n = numel - pos
            full.append((2, pos, n, -(-n // self.AP_RANGE), 0, 0, 0, n, 0, -1, 0, 0, 0, 0, 0, 0))
        blob, blk = bytearray(), 0
        for (kind, off, _n, nblk, d0, d1, R, K, m0, m1, Co, Ci, Cip, Cpad, Cpad_d, Cop) in full:
            blob += struct.pack("<QQq12i", d0, d1, off, kind, blk, R, K, m0, m1, Co, Ci, Cip, Cpad, Cpad_d, Cop)
            blk += nblk
        assert len(blob) == len(full) * self.rt.lib.mmseg_adamw_pack_desc_bytes()
        return torch.frombuffer(blob, dtype=torch.uint8).to(self.rt.device), len(full), blk

    def run(self):
        L, s, code = self.rt.lib, self.rt.stream, self.rt.code
        if self.table is not None:
            L.mmseg_pack_conv3_batched(ptr(self.table), self.n, self.nblocks, code, s)
        if self.gtable is not None:
            L.mmseg_pack_weights_batched(ptr(self.gtable), self.gn, self.gtotal, code, s)
        for d in self.per_layer:
            L.mmseg_pack_weight(*d, code, s)


def _wgrad_ksplit(rows: int, ncols: int, V: int) -> int:
    bn = 64
    tiles = -(-ncols // bn) * -(-rows // (64 if rows % 64 == 0 else 32))
    return max(1, min(-(-TARGET_BLOCKS // tiles), V // 512))


SMALL_IN_V = 4096   # norm_pool.hip knob_small_v(): at or below it InstanceNorm is one launch (stats + apply)


@dataclass
class DySpec:
    """Gradient sources of an InstanceNorm+ReLU output (see mmseg_instnorm_relu_bwd)."""
    p1: Optional[Act] = None
    scale1: float = 1.0
    alpha: Optional[torch.Tensor] = None   # [N][stride] fp32
    alpha_off: int = 0
    alpha_stride: int = 0
    beta: Optional[torch.Tensor] = None    # [N][stride] fp32
    beta_off: int = 0
    beta_stride: int = 0
    pool_dy: Optional[Act] = None
    pool_idx: Optional[torch.Tensor] = None
    # (partials, nchunk): the InstanceNorm-backward partial sums [N][nchunk][C][2] the producer of p1 already
    # emitted (fused head + loss backward), so the partial pass over x and dy is skipped
    part: Optional[Tuple[torch.Tensor, int]] = None
    # > 0: p1 holds p1_nmod samples and sample n reads p1's sample n % p1_nmod -- the fused level's gradient shared
    # by the M modality groups of a grouped block (mmseg_instnorm_relu_bwd_group), instead of an M-fold copy
    p1_nmod: int = 0


class Conv3:
    def __init__(self, rt: Runtime, conv: nn.Conv3d, flat: FlatParams, cin_pad: Optional[int] = None,
                 need_dgrad: bool = True, cout_pad: Optional[int] = None, pad_cols: bool = False):
        """cin_pad: the input tensor's channel count seen by the GEMM (8 x a power of two >= Ci; the extra
        channels meet zero weights).  cout_pad: the same for the data-gradient reduction over Co (its dy
        tensor must hold cout_pad readable channels; pack mode 6 zeroes their weights).
        pad_cols (bias-free convs whose output / input-gradient tensors own cout_pad / cin_pad channels):
        the GEMMs produce the padded column counts (zeros in the padding) and the weight gradient is taken
        over cout_pad rows into a staging buffer, so channel counts like 48 run on the brick kernels."""
        self.rt, self.conv, self.flat = rt, conv, flat
        self.Co, self.Ci = conv.weight.shape[:2]
        self.Cip = cin_pad or self.Ci
        self.Cop = cout_pad or self.Co
        if self.Co % 8 or self.Cip % 8 or self.Cop % 8 or self.Cop < self.Co:
            raise ValueError("conv channels must be multiples of 8")
        if pad_cols and conv.bias is not None:
            raise ValueError("pad_cols: bias-free convs only")
        self.pad_cols = pad_cols
        # column counts the brick kernels take as they are (32- or 48-column tiles) stay unpadded
        tile_ok = lambda c: c % 32 == 0 or c % 48 == 0   # noqa: E731
        self.ncols_f = self.Cop if pad_cols and not tile_ok(self.Co) else self.Co
        self.ncols_d = self.Cip if pad_cols and not tile_ok(self.Ci) else self.Ci
        self.cpg_shift = pow2_shift(self.Cip // 8)
        self.KG = 27 * self.Cip // 8
        self.KGp = round_up(self.KG, 4)
        self.Cpad = _col_tile(self.ncols_f)
        # zeros: the batched pack never writes the K / Cin padding entries
        self.wf = torch.zeros(self.KGp * self.Cpad * 8, dtype=rt.dtype, device=rt.device)
        self.need_dgrad = need_dgrad
        if need_dgrad:
            self.dshift = pow2_shift(self.Cop // 8)
            self.KGd = 27 * self.Cop // 8
            self.KGdp = round_up(self.KGd, 4)
            self.Cpad_d = _col_tile(self.ncols_d)
            self.wd = torch.zeros(self.KGdp * self.Cpad_d * 8, dtype=rt.dtype, device=rt.device)
        # weight gradient over Cop rows (brick kernels need Co % 32 == 0) into a staging [Cop][Ci][27]
        self.wg_stage = (torch.empty(self.Cop * self.Ci * 27, dtype=torch.float32, device=rt.device)
                         if pad_cols and self.Co % 32 and self.Cop % 32 == 0 else None)
        # real channels of the channel-padded K sides (0 = none padded): the brick kernels skip the
        # 32-channel chunks past them
        self.kreal_f = self.Ci if self.Cip > self.Ci else 0
        self.kreal_d = self.Co if self.Cop > self.Co else 0
        self._f8 = None   # (e4m3 weight image, per-output-channel dequant) when the fp8 forward applies

    def fp8_ok(self, x: Act, y: Act) -> bool:
        """Mixed bf16/fp8: this conv's forward runs on e4m3 operands (Runtime.fp8 and the kernel takes the shape)."""
        if not getattr(self.rt, "fp8", False) or self.pad_cols or self.Cip != self.Ci or self.ncols_f != self.Co:
            return False
        return bool(self.rt.lib.mmseg_conv3_fp8_ok(x.N * x.V, self.ncols_f, self.Cpad, self.KG, self.cpg_shift, x.D,
                                                   x.H, x.W, x.ld, y.ld))

    def _fp8_weights(self):
        """e4m3 image of the CURRENT fp32 weights (re-packed every forward, like the bf16 images)."""
        if self._f8 is None:
            self._f8 = (torch.empty(self.KGp * self.Cpad * 8, dtype=torch.uint8, device=self.rt.device),
                        torch.empty(self.Co, dtype=torch.float32, device=self.rt.device))
        w8, dq = self._f8
        self.rt.lib.mmseg_pack_conv3_fp8(ptr(self.conv.weight), self.Co, self.Ci, self.Cip, self.KGp, self.Cpad,
                                         ptr(w8), ptr(dq), self.rt.stream)
        return w8, dq

    def fwd_fp8(self, x: Act, y: Act, norm: Optional[Tuple[torch.Tensor, torch.Tensor]] = None):
        """fwd() / fwd_norm() on e4m3 operands (requires fp8_ok)."""
        w8, dq = self._fp8_weights()
        nm, nr = (ptr(norm[0]), ptr(norm[1])) if norm is not None else (None, None)
        with TIMER.region("conv3_brick6_kernel<BN32,F8>[fp8]", flops=2.0 * x.N * x.V * self.Co * 27 * self.Ci,
                          nbytes=_io_bytes(self.rt, x.N * x.V, self.Cip, self.Co, 27 * self.Cip * self.Co, 1)):
            self.rt.lib.mmseg_conv3_fwd_fp8(x.ptr, x.ld, nm, nr, ptr(w8), ptr(dq), ptr(self.conv.bias), y.ptr, y.ld,
                                            x.N * x.V, self.ncols_f, self.Cpad, self.KG, self.cpg_shift, x.D, x.H,
                                            x.W, self.rt.stream)

    def descs(self):
        w = self.conv.weight
        d = [(ptr(w), ptr(self.wf), 0, self.Co, self.Ci, self.Cip, self.KG, self.KGp, self.Cpad)]
        if self.need_dgrad:
            if self.Cop != self.Co:
                d.append((ptr(w), ptr(self.wd), 6, self.Co, self.Ci, self.Cop, self.KGd, self.KGdp, self.Cpad_d))
            else:
                d.append((ptr(w), ptr(self.wd), 1, self.Co, self.Ci, self.Cip, self.KGd, self.KGdp, self.Cpad_d))
        return d

    def pack(self):
        for d in self.descs():
            self.rt.lib.mmseg_pack_weight(*d, self.rt.code, self.rt.stream)

    def _stem(self, x: Act, y_ld: int) -> bool:
        """First conv on the packed input: K = 27*Ci real taps*channels (stem.hip).  The 48-output-channel stem is
        SwinUNETR's bias-free encoder1 conv only: its weight gradient has no bias term, fused statistics or fused
        norm backward, so a biased 48-channel first conv (a UNet3D / DualEncoder with features[0] = 48) takes the
        implicit-GEMM path."""
        if self.Co == 48 and self.conv.bias is not None:
            return False
        return (not self.need_dgrad and self.Cip == 8
                and bool(self.rt.lib.mmseg_stem_ok(self.Ci, self.Co, x.D, x.H, x.W, x.ld, y_ld)))

    def stats_bricks(self, x: Act, y: Act) -> int:
        """Bricks per sample for which fwd() can emit fused InstanceNorm partials (0 = not available)."""
        if self._stem(x, y.ld):
            # the stem's epilogue can emit its output's statistics per 64-voxel slice, but that measured slower
            # (stem +14.5 us and the slice merge 105 us per launch against a 20 + 5 us statistics pass, rocprofv3
            # r02h): the statistics pass runs (mmseg_stem_fwd_stats stays in the ABI)
            return 0
        return self.rt.lib.mmseg_conv3_stats_bricks(x.N * x.V, self.Co, self.Cpad, self.KG, self.cpg_shift, x.D, x.H,
                                                    x.W, x.ld, y.ld, self.rt.code)

    def fwd(self, x: Act, y: Act, stats_part: Optional[torch.Tensor] = None):
        if stats_part is not None and self._stem(x, y.ld):
            with TIMER.region("stem_fwd_kernel", flops=2.0 * x.N * x.V * self.Co * 27 * self.Ci,
                              nbytes=_io_bytes(self.rt, x.N * x.V, 8, self.Co, 27 * self.Ci * self.Co, 4)):
                self.rt.lib.mmseg_stem_fwd_stats(x.ptr, x.ld, self.Ci, ptr(self.conv.weight), ptr(self.conv.bias),
                                                 y.ptr, y.ld, x.N, x.D, x.H, x.W, self.Co, ptr(stats_part),
                                                 self.rt.code, self.rt.stream)
            return
        if stats_part is not None:
            with TIMER.region(_gemm_name(self.rt, self.Co, "conv3"), flops=2.0 * x.N * x.V * self.Co * 27 * self.Ci,
                              nbytes=_io_bytes(self.rt, x.N * x.V, self.Ci, self.Co, 27 * self.Ci * self.Co)):
                self.rt.lib.mmseg_conv_gemm_ex(x.ptr, x.ld, ptr(self.wf), ptr(self.conv.bias), y.ptr, y.ld, None,
                                               MODE_CONV3, x.N * x.V, self.Co, self.Cpad, self.KG, self.cpg_shift,
                                               x.D, x.H, x.W, 1, ptr(stats_part), self.kreal_f, self.rt.code,
                                               self.rt.stream)
            return
        if self._stem(x, y.ld):
            with TIMER.region("stem_fwd_kernel", flops=2.0 * x.N * x.V * self.Co * 27 * self.Ci,
                              nbytes=_io_bytes(self.rt, x.N * x.V, 8, self.Co, 27 * self.Ci * self.Co, 4)):
                self.rt.lib.mmseg_stem_fwd(x.ptr, x.ld, self.Ci, ptr(self.conv.weight), ptr(self.conv.bias), y.ptr,
                                           y.ld, x.N, x.D, x.H, x.W, self.Co, self.rt.code, self.rt.stream)
            return
        if self.fp8_ok(x, y):
            self.fwd_fp8(x, y)
            return
        M = x.N * x.V
        nc = self.ncols_f
        ks = self.rt.lib.mmseg_conv3_splits(M, nc, self.Cpad, self.KG, self.cpg_shift, x.D, x.H, x.W, x.ld, y.ld,
                                            self.rt.code)
        ws = self.rt.ws(ks * M * nc) if ks > 1 else None
        with TIMER.region(_gemm_name(self.rt, nc, "conv3"), flops=2.0 * M * self.Co * 27 * self.Ci,
                          nbytes=_io_bytes(self.rt, M, self.Cip, self.Co, 27 * self.Cip * self.Co)):
            # (an output owning its padded rows is written whole: Act.wcols, mmseg_conv_gemm_zw)
            self.rt.lib.mmseg_conv_gemm_zw(x.ptr, x.ld, ptr(self.wf), ptr(self.conv.bias), y.ptr, y.ld, ptr(ws),
                                           MODE_CONV3, M, nc, self.Cpad, self.KG, self.cpg_shift, x.D, x.H, x.W, ks,
                                           self.kreal_f, _zcols(y, nc), self.rt.code, self.rt.stream)

    def norm_ok(self, x: Act, y: Act) -> bool:
        """True when this conv can take its input as the PRE-norm activation of an InstanceNorm + ReLU and apply
        it on staging, forward and weight gradient (fwd_norm / bwd(norm=...)): the brick5 / brick2 kernels."""
        L, code = self.rt.lib, self.rt.code
        return (self.need_dgrad and self.wg_stage is None and self.Cip == self.Ci and self.ncols_f == self.Co
                and not self._stem(x, y.ld)
                and bool(L.mmseg_conv3_norm_ok(x.N * x.V, self.ncols_f, self.Cpad, self.KG, self.cpg_shift, x.D,
                                               x.H, x.W, x.ld, y.ld, code))
                and bool(L.mmseg_conv3_wgrad_norm_ok(x.N * x.V, self.Co, self.Cip, self.Ci, self.cpg_shift, x.D,
                                                     x.H, x.W, y.ld, x.ld, code)))

    def fwd_norm(self, x: Act, mean: torch.Tensor, rstd: torch.Tensor, y: Act):
        """fwd() of relu(InstanceNorm(x)) with x the pre-norm activation (requires norm_ok)."""
        if self.fp8_ok(x, y):
            self.fwd_fp8(x, y, norm=(mean, rstd))
            return
        with TIMER.region(_gemm_name(self.rt, self.ncols_f, "conv3"), flops=2.0 * x.N * x.V * self.Co * 27 * self.Ci,
                          nbytes=_io_bytes(self.rt, x.N * x.V, self.Cip, self.Co, 27 * self.Cip * self.Co)):
            self.rt.lib.mmseg_conv3_fwd_norm(x.ptr, x.ld, ptr(mean), ptr(rstd), ptr(self.wf), ptr(self.conv.bias),
                                             y.ptr, y.ld, x.N * x.V, self.ncols_f, self.Cpad, self.KG,
                                             self.cpg_shift, x.D, x.H, x.W, self.rt.code, self.rt.stream)

    def _part(self, nfloats: int, own: bool = False) -> torch.Tensor:
        """Split partials of this layer's weight gradient: the shared scratch, or with the side-stream reduce
        (Runtime.async_wred) or a deferred one (own: Runtime.defer_wred) a buffer of the layer's own, since its
        reduce may still run while later kernels take scratch (the partials of a whole backward, ~1.2 GB for the
        96^3 DualEncoder, fit HBM many times over)."""
        if not self.rt.async_wred and not own:
            return self.rt.ws(nfloats)
        if own:
            return self.rt.own_part(self, nfloats)
        buf = getattr(self, "_wpart", None)
        if buf is None or buf.numel() < nfloats:
            buf = self._wpart = torch.empty(int(nfloats), dtype=torch.float32, device=self.rt.device)
        return buf

    def _reduce_after(self, fn) -> None:
        """Run fn(stream) -- the split reduce, the staging copy and the DP readiness mark -- after the weight-gradient
        kernel: on the side stream, beside this layer's data-gradient kernel (the mark then records the DP bucket
        event there; bwd joins the side stream before it returns), or in line."""
        if self.rt.async_wred:
            with self.rt.fork_side():
                fn(self.rt.stream)
        else:
            fn(self.rt.stream)

    def bwd(self, *args, **kw):
        try:
            return self._bwd(*args, **kw)
        finally:
            self.rt.join_side()

    def _bwd(self, x: Act, dy: Act, dx: Optional[Act], accumulate: bool,
            norm: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
            inp: Optional[Tuple[Act, torch.Tensor, torch.Tensor]] = None,
            inb: Optional[Tuple[Act, torch.Tensor, torch.Tensor, torch.Tensor]] = None):
        """norm = (mean, rstd): x is the pre-norm activation of an InstanceNorm + ReLU applied on staging by the
        weight-gradient kernel (see fwd_norm).  inp = (pre-norm x, mean, rstd) of the InstanceNorm + ReLU whose
        output gradient dx is: when the data-gradient kernel can, it also writes that backward's partial sums;
        returns (partials, chunks) for DySpec.part, or None.  inb = (pre-norm x, mean, rstd, coef) (stem only, see
        stem_inb_ok): dy is the gradient of that norm's OUTPUT and the stem weight gradient applies the norm's
        backward while staging it (mmseg_stem_wgrad_inb)."""
        L, s, code = self.rt.lib, self.rt.stream, self.rt.code
        V = x.N * x.V
        if dx is None and norm is None and (inb is not None or self._stem(x, dy.ld)):
            # 1,024 splits: one round of resident blocks at 96^3 B=2 and half the partials of 2,048 (r02 stembench:
            # 42 + 12.8 us against 44 + 19.7 us with the reduce)
            ks = L.mmseg_stem_wgrad_splits(x.N, x.D, x.H, x.W, 1024)
            kp = L.mmseg_stem_kp(self.Ci)
            defer = self.rt.defer_wred(self.flat)
            part = self._part(ks * self.Co * kp + ks * self.Co, own=defer)
            has_b = self.conv.bias is not None
            bpart = part.data_ptr() + ks * self.Co * kp * 4 if has_b else None
            with TIMER.region("stem_wgrad_kernel", flops=2.0 * V * self.Co * 27 * self.Ci,
                              nbytes=_io_bytes(self.rt, V, 8, self.Co, 27 * self.Ci * self.Co, 4)):
                if inb is not None:
                    xi, im, ir, cf = inb
                    L.mmseg_stem_wgrad_inb(dy.ptr, dy.ld, x.ptr, x.ld, self.Ci, xi.ptr, xi.ld, ptr(im), ptr(ir),
                                           ptr(cf), ptr(part), bpart, x.N, x.D, x.H, x.W, self.Co, ks, code, s)
                else:
                    L.mmseg_stem_wgrad(dy.ptr, dy.ld, x.ptr, x.ld, self.Ci, ptr(part), bpart, x.N, x.D, x.H, x.W,
                                       self.Co, ks, code, s)
            (L.mmseg_wgrad_reduce_defer if defer else L.mmseg_wgrad_reduce)(
                ptr(part), ptr(self.flat.grad(self.conv.weight)), bpart,
                ptr(self.flat.grad(self.conv.bias)) if has_b else None, self.Co, kp, ks, self.Ci, self.Ci, 27,
                int(accumulate), s)
            self.flat.mark(*[p for p in (self.conv.weight, self.conv.bias) if p is not None])
            return
        rows = self.Cop if self.wg_stage is not None else self.Co
        wsf = L.mmseg_conv3_wgrad_ws_floats(V, rows, self.Cip, self.Ci, self.cpg_shift, x.D, x.H, x.W, dy.ld,
                                            x.ld, code)
        # a batched backward queues the split reduce (its partials then need a buffer of their own); not with a
        # staging buffer, whose copy into the arena must follow the reduce
        defer = wsf > 0 and self.wg_stage is None and self.rt.defer_wred(self.flat)
        ws = self._part(wsf, own=defer) if wsf > 0 else None
        wgrad = self.flat.grad(self.conv.weight)
        nm, nr = (ptr(norm[0]), ptr(norm[1])) if norm is not None else (None, None)
        args = (dy.ptr, dy.ld, x.ptr, x.ld, nm, nr, ptr(self.wg_stage) if self.wg_stage is not None else ptr(wgrad),
                ptr(self.flat.grad(self.conv.bias)) if self.conv.bias is not None else None, rows, self.Cip, self.Ci,
                self.cpg_shift, V, x.D, x.H, x.W, ptr(ws), wsf, int(accumulate) if self.wg_stage is None else 0)
        # the kernel and its split reduce are timed separately (the roofline family is the kernel alone, as in
        # the rocprofv3 trace)
        # the staged gradient's last 16 rows are output-channel padding (48 of 64): the 64-row kernel skips them
        pad16 = 8 if (self.wg_stage is not None and rows - self.Co == 16) else 0

        def wkernel(s1):
            with TIMER.region(_gemm_name(self.rt, 0, "conv3"), flops=2.0 * V * self.Co * 27 * self.Ci,
                              nbytes=_io_bytes(self.rt, V, self.Cip, self.Co, 27 * self.Cip * self.Co, 4)):
                L.mmseg_conv3_wgrad_ex(*args, 1 | pad16, code, s1)

        # (the weight gradient beside the data gradient on a side stream measured slower: DESIGN (d) round 4)
        wkernel(s)

        def reduce(s2):
            with TIMER.region("wgrad_reduce_kernel"):
                L.mmseg_conv3_wgrad_ex(*args, 6 if defer else 2, code, s2)
            if self.wg_stage is not None:     # rows [0, Co) of the staging are the gradient's storage order
                n = wgrad.numel()
                if accumulate:
                    L.mmseg_add(ptr(wgrad), ptr(self.wg_stage), ptr(wgrad), n, 0, s2)
                else:
                    wgrad.view(-1).copy_(self.wg_stage[:n])
            self.flat.mark(*[p for p in (self.conv.weight, self.conv.bias) if p is not None])
        if wsf > 0:
            self._reduce_after(reduce)
        else:
            reduce(s)
        if dx is not None:
            # dx = (lo, hi): columns [0, lo.C) into lo, the rest into hi (two dense tensors, mmseg_conv_gemm_split)
            split = isinstance(dx, tuple)
            d0 = dx[0] if split else dx
            M = V
            nc = self.ncols_d
            ks = L.mmseg_conv3_splits(M, nc, self.Cpad_d, self.KGd, self.dshift, x.D, x.H, x.W, dy.ld, d0.ld, code)
            ws = self.rt.ws(ks * M * nc) if ks > 1 else None
            with TIMER.region(_gemm_name(self.rt, nc, "conv3"), flops=2.0 * M * self.Co * 27 * self.Ci,
                              nbytes=_io_bytes(self.rt, M, self.Co, self.Cip, 27 * self.Cip * self.Co)):
                nch = 0
                if inp is not None and not split and ks == 1 and os.environ.get("MMSEG_DGRAD_IN_PART", "1") != "0":
                    nch = L.mmseg_conv3_dgrad_in_chunks(M, nc, self.Cpad_d, self.KGd, self.dshift, x.D, x.H, x.W,
                                                        dy.ld, dx.ld, code)
                if nch:
                    xi, im, ir = inp
                    size = x.N * nch * nc * 2
                    if getattr(self, "_inpart", None) is None or self._inpart.numel() != size:
                        self._inpart = torch.empty(size, dtype=torch.float32, device=self.rt.device)
                    L.mmseg_conv3_dgrad_in(dy.ptr, dy.ld, ptr(self.wd), dx.ptr, dx.ld, M, nc, self.Cpad_d, self.KGd,
                                           self.dshift, x.D, x.H, x.W, xi.ptr, xi.ld, ptr(im), ptr(ir),
                                           ptr(self._inpart), code, s)
                    return self._inpart, nch
                if split:
                    L.mmseg_conv_gemm_split(dy.ptr, dy.ld, ptr(self.wd), None, d0.ptr, d0.ld, dx[1].ptr, dx[1].ld,
                                            d0.C, ptr(ws), MODE_CONV3, M, nc, self.Cpad_d, self.KGd, self.dshift, x.D,
                                            x.H, x.W, ks, self.kreal_d, code, s)
                else:
                    L.mmseg_conv_gemm_zw(dy.ptr, dy.ld, ptr(self.wd), None, dx.ptr, dx.ld, ptr(ws), MODE_CONV3, M,
                                         nc, self.Cpad_d, self.KGd, self.dshift, x.D, x.H, x.W, ks, self.kreal_d,
                                         _zcols(dx, nc), code, s)


class ConvT2:
    def __init__(self, rt: Runtime, up: nn.ConvTranspose3d, flat: FlatParams, cout_pad: Optional[int] = None):
        """cout_pad: channels of dy read by the data-gradient / weight-gradient gathers (8 x a power of two
        >= Co; pack mode 7 zeroes their weights, the reduce drops their weight-gradient columns)."""
        self.rt, self.up, self.flat = rt, up, flat
        self.Ci, self.Co = up.weight.shape[:2]
        self.Cop = cout_pad or self.Co
        if self.Ci % 8 or self.Co % 8 or self.Cop % 8 or self.Cop < self.Co:
            raise ValueError("transposed-conv channels must be multiples of 8")
        self.KG = self.Ci // 8
        self.KGp = round_up(self.KG, 4)
        self.Cpad = _col_tile(8 * self.Co)
        self.wf = torch.empty(self.KGp * self.Cpad * 8, dtype=rt.dtype, device=rt.device)
        self.dshift = pow2_shift(self.Cop // 8)
        self.KGd = self.Cop  # 8 taps x Cop/8 groups
        self.KGdp = round_up(self.KGd, 4)
        self.Cpad_d = _col_tile(self.Ci)
        self.wd = torch.empty(self.KGdp * self.Cpad_d * 8, dtype=rt.dtype, device=rt.device)

    def descs(self):
        w = self.up.weight
        if self.Cop != self.Co:
            dd = (ptr(w), ptr(self.wd), 7, self.Co, self.Ci, self.Cop, self.KGd, self.KGdp, self.Cpad_d)
        else:
            dd = (ptr(w), ptr(self.wd), 5, self.Co, self.Ci, self.Ci, self.KGd, self.KGdp, self.Cpad_d)
        return [(ptr(w), ptr(self.wf), 4, self.Co, self.Ci, self.Ci, self.KG, self.KGp, self.Cpad), dd]

    def pack(self):
        for d in self.descs():
            self.rt.lib.mmseg_pack_weight(*d, self.rt.code, self.rt.stream)

    def fwd(self, x: Act, y: Act):
        M = x.N * x.V
        ncols = 8 * self.Co
        ks = _gemm_ksplit(M, ncols, self.KG)
        ws = self.rt.ws(ks * M * ncols) if ks > 1 else None
        with TIMER.region(_gemm_name(self.rt, 0, "convT"), flops=2.0 * M * self.Ci * 8 * self.Co,
                          nbytes=_io_bytes(self.rt, M, self.Ci, 8 * self.Co, 8 * self.Ci * self.Co)):
            self.rt.lib.mmseg_conv_gemm(x.ptr, x.ld, ptr(self.wf), ptr(self.up.bias), y.ptr, y.ld, ptr(ws),
                                        MODE_CONVT_FWD, M, ncols, self.Cpad, self.KG, 0, x.D, x.H, x.W, ks,
                                        self.rt.code, self.rt.stream)

    def bwd(self, x: Act, dy: Act, dx: Optional[Act], accumulate: bool):
        """x: input grid (D,H,W); dy: output grid (2D,2H,2W)."""
        L, s, code = self.rt.lib, self.rt.stream, self.rt.code
        V = x.N * x.V
        ncols = 8 * self.Cop
        ks = L.mmseg_wgrad_splits(V, _wgrad_ksplit(self.Ci, ncols, V))
        # bias gradient: column sums of the gathered dy tile emitted by the weight-gradient kernel itself
        # ([ks][8 Cop] after the weight partials, folded over (split, tap)), so dy is read once
        fused_bias = self.up.bias is not None and self.Cop == self.Co
        # (the unfused bias sums reuse the partial buffer after the reduce: that reduce stays in line)
        defer = (fused_bias or self.up.bias is None) and self.rt.defer_wred(self.flat)
        nfl = max(ks * self.Ci * ncols + (ks * ncols if fused_bias else 0), 256 * self.Co)
        part = _own_part(self, self.rt, nfl) if defer else self.rt.ws(nfl)
        bpart = part.data_ptr() + ks * self.Ci * ncols * 4 if fused_bias else None
        with TIMER.region(_gemm_name(self.rt, 0, "convT"), flops=2.0 * V * self.Ci * 8 * self.Co,
                          nbytes=_io_bytes(self.rt, V, self.Ci, 8 * self.Co, 8 * self.Ci * self.Co, 4)):
            L.mmseg_wgrad(x.ptr, x.ld, dy.ptr, dy.ld, ptr(part), bpart, MODE_CONVT_DGRAD, self.Ci, ncols,
                          self.dshift, V, x.D, x.H, x.W, ks, code, s)
        (L.mmseg_wgrad_reduce_defer if defer else L.mmseg_wgrad_reduce)(
            ptr(part), ptr(self.flat.grad(self.up.weight)), None, None, self.Ci, ncols, ks, self.Cop, self.Co, 8,
            int(accumulate), s)
        if fused_bias:
            L.mmseg_colsum_reduce(bpart, 8 * ks, self.Co, ptr(self.flat.grad(self.up.bias)), int(accumulate), s)
        elif self.up.bias is not None:
            L.mmseg_colsum(dy.ptr, dy.ld, self.Co, dy.N * dy.V, ptr(part), 256, ptr(self.flat.grad(self.up.bias)),
                           int(accumulate), code, s)
        self.flat.mark(*[p for p in (self.up.weight, self.up.bias) if p is not None])
        if dx is not None:
            ks = _gemm_ksplit(V, self.Ci, self.KGd)
            ws = self.rt.ws(ks * V * self.Ci) if ks > 1 else None
            with TIMER.region(_gemm_name(self.rt, 0, "convT"), flops=2.0 * V * self.Ci * 8 * self.Co,
                              nbytes=_io_bytes(self.rt, V, 8 * self.Co, self.Ci, 8 * self.Ci * self.Co)):
                L.mmseg_conv_gemm(dy.ptr, dy.ld, ptr(self.wd), None, dx.ptr, dx.ld, ptr(ws), MODE_CONVT_DGRAD, V,
                                  self.Ci, self.Cpad_d, self.KGd, self.dshift, x.D, x.H, x.W, ks, code, s)


class Point:
    """1x1x1 Conv3d on NDHWC (the DualEncoder concat-fusion projection)."""

    def __init__(self, rt: Runtime, conv: nn.Conv3d, flat: FlatParams):
        self.rt, self.conv, self.flat = rt, conv, flat
        self.Co, self.Ci = conv.weight.shape[:2]
        self.KG, self.KGp, self.Cpad = self.Ci // 8, round_up(self.Ci // 8, 4), _col_tile(self.Co)
        self.KGd, self.KGdp, self.Cpad_d = self.Co // 8, round_up(self.Co // 8, 4), _col_tile(self.Ci)
        self.wf = torch.empty(self.KGp * self.Cpad * 8, dtype=rt.dtype, device=rt.device)
        self.wd = torch.empty(self.KGdp * self.Cpad_d * 8, dtype=rt.dtype, device=rt.device)

    def descs(self):
        w = self.conv.weight
        return [(ptr(w), ptr(self.wf), 2, self.Co, self.Ci, self.Ci, self.KG, self.KGp, self.Cpad),
                (ptr(w), ptr(self.wd), 3, self.Co, self.Ci, self.Ci, self.KGd, self.KGdp, self.Cpad_d)]

    def pack(self):
        for d in self.descs():
            self.rt.lib.mmseg_pack_weight(*d, self.rt.code, self.rt.stream)

    def fwd(self, x: Act, y: Act):
        M = x.N * x.V
        with TIMER.region(_gemm_name(self.rt, 0, "point"), flops=2.0 * M * self.Ci * self.Co,
                          nbytes=_io_bytes(self.rt, M, self.Ci, self.Co, self.Ci * self.Co)):
            self.rt.lib.mmseg_conv_gemm(x.ptr, x.ld, ptr(self.wf), ptr(self.conv.bias), y.ptr, y.ld, None, MODE_POINT,
                                        M, self.Co, self.Cpad, self.KG, 0, x.D, x.H, x.W, 1, self.rt.code,
                                        self.rt.stream)

    def bwd(self, x: Act, dy: Act, dx: Optional[Act], accumulate: bool):
        L, s, code = self.rt.lib, self.rt.stream, self.rt.code
        V = x.N * x.V
        ks = L.mmseg_wgrad_splits(V, _wgrad_ksplit(self.Co, self.Ci, V))
        defer = self.rt.defer_wred(self.flat)
        nfl = ks * self.Co * self.Ci + ks * self.Co
        part = _own_part(self, self.rt, nfl) if defer else self.rt.ws(nfl)
        bpart = part.data_ptr() + ks * self.Co * self.Ci * 4
        with TIMER.region(_gemm_name(self.rt, 0, "point"), flops=2.0 * V * self.Ci * self.Co,
                          nbytes=_io_bytes(self.rt, V, self.Ci, self.Co, self.Ci * self.Co, 4)):
            L.mmseg_wgrad(dy.ptr, dy.ld, x.ptr, x.ld, ptr(part), bpart, MODE_POINT, self.Co, self.Ci, 0, V, x.D, x.H,
                          x.W, ks, code, s)
        (L.mmseg_wgrad_reduce_defer if defer else L.mmseg_wgrad_reduce)(
            ptr(part), ptr(self.flat.grad(self.conv.weight)), bpart, ptr(self.flat.grad(self.conv.bias)), self.Co,
            self.Ci, ks, self.Ci, self.Ci, 1, int(accumulate), s)
        self.flat.mark(self.conv.weight, self.conv.bias)
        if dx is not None:
            with TIMER.region(_gemm_name(self.rt, 0, "point"), flops=2.0 * V * self.Ci * self.Co,
                              nbytes=_io_bytes(self.rt, V, self.Co, self.Ci, self.Ci * self.Co)):
                L.mmseg_conv_gemm(dy.ptr, dy.ld, ptr(self.wd), None, dx.ptr, dx.ld, None, MODE_POINT, V, self.Ci,
                                  self.Cpad_d, self.KGd, 0, x.D, x.H, x.W, 1, code, s)


class Block:
    """ConvBlock3D: conv1 -> IN -> ReLU -> conv2 -> IN -> ReLU (reference unet.py:53-60)."""

    def __init__(self, rt: Runtime, module: nn.Module, flat: FlatParams, cin_pad: Optional[int] = None,
                 need_dgrad: bool = True):
        self.rt = rt
        self.c1 = Conv3(rt, module.conv1, flat, cin_pad=cin_pad, need_dgrad=need_dgrad)
        self.c2 = Conv3(rt, module.conv2, flat)
        self.Co = self.c1.Co
        self.shape = None
        # defer_out: the block's last InstanceNorm + ReLU is applied by its consumers on load (DualEncoder mean /
        # add fusion: maxpool + fusion read x2 and the statistics), so `out` is not written by fwd();
        # materialize_out() writes it when someone needs it (return_features)
        self.defer_out = False

    def descs(self):
        return self.c1.descs() + self.c2.descs()

    def pack(self):
        self.c1.pack()
        self.c2.pack()

    def setup(self, N, D, H, W):
        if self.shape == (N, D, H, W):
            return
        self.shape = (N, D, H, W)
        rt, C = self.rt, self.Co
        self.x1 = rt.act(N, D, H, W, C)
        self.y1 = rt.act(N, D, H, W, C)
        self.x2 = rt.act(N, D, H, W, C)
        self.stats = torch.empty(4, N * C, dtype=torch.float32, device=rt.device)  # m1, r1, m2, r2
        self.nb = None   # fused-statistics bricks per sample of (conv1, conv2), set on the first forward
        # conv1's InstanceNorm + ReLU applied by conv2's kernels on staging (y1 never written): the 96^3 32 -> 32
        # layers (brick5 forward, brick2 weight gradient)
        self.norm1_ok = None
        self.defer1 = False

    def _norm_fwd(self, x: Act, y: Act, m: torch.Tensor, r: torch.Tensor, part=None, nb: int = 0):
        L, s, code = self.rt.lib, self.rt.stream, self.rt.code
        if part is not None:
            L.mmseg_instnorm_stats_bricks(ptr(part), x.N, x.C, nb, x.V // nb, IN_EPS, ptr(m), x.C, ptr(r), s)
            L.mmseg_instnorm_relu_fwd(x.ptr, x.ld, y.ptr, y.ld, x.N, x.V, x.C, ptr(m), ptr(r), code, s)
        else:
            ws = self.rt.ws(L.mmseg_instnorm_ws_floats(x.N, x.V, x.C))
            L.mmseg_instnorm_fwd(x.ptr, x.ld, y.ptr, y.ld, x.N, x.V, x.C, IN_EPS, ptr(m), x.C, ptr(r), 1, ptr(ws),
                                 code, s)

    def _norm_bwd(self, x: Act, m: torch.Tensor, r: torch.Tensor, dy: DySpec, dx: Act):
        L, s, code = self.rt.lib, self.rt.stream, self.rt.code
        ws = self.rt.ws(L.mmseg_instnorm_ws_floats(x.N, x.V, x.C))
        p1 = dy.p1
        es = 4
        alpha = None if dy.alpha is None else dy.alpha.data_ptr() + dy.alpha_off * es
        beta = None if dy.beta is None else dy.beta.data_ptr() + dy.beta_off * es
        if dy.p1_nmod:
            assert dy.part is None and alpha is None and beta is None and p1 is not None
            L.mmseg_instnorm_relu_bwd_group(x.ptr, x.ld, ptr(m), ptr(r), p1.ptr, p1.ld, dy.scale1, dy.p1_nmod,
                                            dy.pool_dy.ptr if dy.pool_dy is not None else None,
                                            dy.pool_dy.ld if dy.pool_dy is not None else 0, ptr(dy.pool_idx),
                                            dx.ptr, dx.ld, x.N, x.D, x.H, x.W, x.C, ptr(ws), code, s)
            return
        if dy.part is not None:
            assert dy.pool_dy is None and alpha is None and beta is None
            part, nch = dy.part
            L.mmseg_instnorm_bwd_part(x.ptr, x.ld, ptr(m), ptr(r), p1.ptr, p1.ld, dy.scale1, None, 0, None, 0,
                                      None, 0, None, dx.ptr, dx.ld, x.N, x.D, x.H, x.W, x.C, 1, ptr(part), nch,
                                      ptr(ws), code, s)
            return
        L.mmseg_instnorm_relu_bwd(x.ptr, x.ld, ptr(m), ptr(r),
                                  p1.ptr if p1 is not None else None, p1.ld if p1 is not None else 0, dy.scale1,
                                  alpha, dy.alpha_stride, beta, dy.beta_stride,
                                  dy.pool_dy.ptr if dy.pool_dy is not None else None,
                                  dy.pool_dy.ld if dy.pool_dy is not None else 0, ptr(dy.pool_idx),
                                  dx.ptr, dx.ld, x.N, x.D, x.H, x.W, x.C, ptr(ws), code, s)

    def fwd(self, xin: Act, out: Act):
        self.setup(xin.N, xin.D, xin.H, xin.W)
        st = self.stats
        if self.nb is None:
            self.nb = (self.c1.stats_bricks(xin, self.x1), self.c2.stats_bricks(self.y1, self.x2))
            n = max(self.nb)
            self.part = torch.empty(xin.N * n * self.Co * 2, dtype=torch.float32, device=self.rt.device) if n else None
        p1 = self.part if self.nb[0] else None
        p2 = self.part if self.nb[1] else None
        if self.norm1_ok is None:
            self.norm1_ok = not self.nb[1] and self.c2.norm_ok(self.x1, self.x2)
        self.defer1 = self.norm1_ok and os.environ.get("MMSEG_DEFER_CONV_NORM", "1") != "0"   # per forward (A/B)
        self.c1.fwd(xin, self.x1, stats_part=p1)
        if self.defer1:
            self._norm_stats(self.x1, st[0], st[1], p1, self.nb[0])
            self.c2.fwd_norm(self.x1, st[0], st[1], self.x2)
        else:
            self._norm_fwd(self.x1, self.y1, st[0], st[1], p1, self.nb[0])
            self.c2.fwd(self.y1, self.x2, stats_part=p2)
        if self.defer_out:
            self._norm_stats(self.x2, st[2], st[3], p2, self.nb[1])
        else:
            self._norm_fwd(self.x2, out, st[2], st[3], p2, self.nb[1])

    def _norm_stats(self, x: Act, m: torch.Tensor, r: torch.Tensor, part=None, nb: int = 0):
        L, s, code = self.rt.lib, self.rt.stream, self.rt.code
        if part is not None:
            L.mmseg_instnorm_stats_bricks(ptr(part), x.N, x.C, nb, x.V // nb, IN_EPS, ptr(m), x.C, ptr(r), s)
        else:
            ws = self.rt.ws(L.mmseg_instnorm_ws_floats(x.N, x.V, x.C))
            L.mmseg_instnorm_stats(x.ptr, x.ld, x.N, x.V, x.C, IN_EPS, ptr(m), x.C, ptr(r), ptr(ws), code, s)

    def out_stats(self):
        """(pre-norm x2, mean, rstd) of the block's output InstanceNorm (for consumers of a deferred output)."""
        return self.x2, self.stats[2], self.stats[3]

    def materialize_out(self, out: Act):
        L = self.rt.lib
        L.mmseg_instnorm_relu_fwd(self.x2.ptr, self.x2.ld, out.ptr, out.ld, self.x2.N, self.x2.V, self.x2.C,
                                  ptr(self.stats[2]), ptr(self.stats[3]), self.rt.code, self.rt.stream)

    def bwd(self, xin: Act, dy: Optional[DySpec], dxin: Optional[Act], accumulate: bool, out_done: bool = False):
        """out_done: the output InstanceNorm's backward already ran (grouped over the modalities, in place over x2)."""
        st = self.stats
        g2 = self.x2                      # in place over x2
        if not out_done:
            self._norm_bwd(self.x2, st[2], st[3], dy, g2)
        dy1 = self.y1                     # conv2 wgrad reads y1 before dgrad overwrites it
        # conv2's data gradient may also sum conv1's InstanceNorm-backward partials (brick5 shapes)
        inp = (self.x1, st[0], st[1])
        if self.defer1:                   # (y1 was never written: the weight gradient normalises x1 itself)
            part = self.c2.bwd(self.x1, g2, dy1, accumulate, norm=(st[0], st[1]), inp=inp)
        else:
            part = self.c2.bwd(self.y1, g2, dy1, accumulate, inp=inp)
        g1 = self.x1
        if dxin is None and self._stem_inb(xin):
            # conv1 is the stem and its weight gradient is the only reader of conv1's InstanceNorm input gradient:
            # only the norm's coefficients are formed here, the stem applies the backward while staging dy1
            L, s, code = self.rt.lib, self.rt.stream, self.rt.code
            x1 = self.x1
            if getattr(self, "_coef", None) is None:
                self._coef = torch.empty(x1.N * x1.C * 2, dtype=torch.float32, device=self.rt.device)
            ws = self.rt.ws(L.mmseg_instnorm_ws_floats(x1.N, x1.V, x1.C)) if part is None else None
            L.mmseg_instnorm_bwd_coef(x1.ptr, x1.ld, ptr(st[0]), ptr(st[1]), dy1.ptr, dy1.ld, x1.N, x1.D, x1.H,
                                      x1.W, x1.C, 1, ptr(part[0]) if part else None, part[1] if part else 0,
                                      ptr(self._coef), ptr(ws), code, s)
            self.c1.bwd(xin, dy1, None, accumulate, inb=(x1, st[0], st[1], self._coef))
            return
        self._norm_bwd(self.x1, st[0], st[1], DySpec(p1=dy1, part=part), g1)
        self.c1.bwd(xin, g1, dxin, accumulate)

    def _stem_inb(self, xin: Act) -> bool:
        """conv1's InstanceNorm backward applied inside the stem weight gradient (no input gradient written):
        conv1 takes the stem path, has no data gradient, and the volume is above the one-launch small-IN size
        (whose backward sums in another order)."""
        return (not self.c1.need_dgrad and self.c1.Co != 48 and self.x1.V > SMALL_IN_V
                and self.c1._stem(xin, self.x1.ld))


class ConvGroup:
    """G same-shape Conv3 layers (the M modality encoders' copies of one layer) run as ONE launch over the G x N
    samples of a combined activation (mmseg_conv_gemm_group / mmseg_conv3_wgrad_group): group g reads its own
    packed weights (the layers' images are laid out at a fixed stride, DualEncoderProgram) and bias, and writes its
    own gradients (the encoders' parameters sit at a fixed stride in the flat arena).  At the 12^3 / 6^3 levels a
    modality's launch fills a fraction of the CUs; the grouped one does twice (M = 2) the work per launch."""

    def __init__(self, convs: List["Conv3"]):
        self.convs = list(convs)
        self.G = len(self.convs)
        c0 = self.convs[0]
        self.c0, self.rt, self.flat = c0, c0.rt, c0.flat

        def stride(get, es):
            p = [get(c) for c in self.convs]
            d = {(p[i + 1] - p[i]) for i in range(len(p) - 1)}
            if len(d) != 1 or next(iter(d)) % es:
                return None
            return next(iter(d)) // es
        es = self.rt.dtype.itemsize
        self.w_gs = stride(lambda c: ptr(c.wf), es)
        self.wd_gs = stride(lambda c: ptr(c.wd), es) if c0.need_dgrad else 0
        fl = self.flat
        self.b_gs = stride(lambda c: ptr(c.conv.bias), 4) if c0.conv.bias is not None else 0
        self.gw_gs = stride(lambda c: ptr(fl.grad(c.conv.weight)), 4)
        self.gb_gs = stride(lambda c: ptr(fl.grad(c.conv.bias)), 4) if c0.conv.bias is not None else 0
        self.layout_ok = (None not in (self.w_gs, self.wd_gs, self.b_gs, self.gw_gs, self.gb_gs)
                          and all(c.wg_stage is None and c.Cip == c.Ci and not c.pad_cols and c.need_dgrad
                                  for c in self.convs))

    def ok(self, x: Act, y: Act) -> bool:
        """x / y: the combined (G x N sample) input and output of the layer's forward."""
        if not self.layout_ok:
            return False
        c, L, code = self.c0, self.rt.lib, self.rt.code
        M = x.N * x.V
        return (bool(L.mmseg_conv3_group_ok(M, c.ncols_f, c.Cpad, c.KG, c.cpg_shift, x.D, x.H, x.W, x.ld, y.ld, code))
                and bool(L.mmseg_conv3_group_ok(M, c.ncols_d, c.Cpad_d, c.KGd, c.dshift, x.D, x.H, x.W, y.ld, x.ld,
                                                code))
                and bool(L.mmseg_conv3_wgrad_group_ok(M, c.Co, c.Cip, c.Ci, c.cpg_shift, x.D, x.H, x.W, y.ld, x.ld,
                                                      code)))

    def stats_bricks(self, x: Act, y: Act) -> int:
        """Bricks per sample for which fwd() can emit fused InstanceNorm partials (0 = not available)."""
        c = self.c0
        return self.rt.lib.mmseg_conv3_group_stats_bricks(x.N * x.V, c.ncols_f, c.Cpad, c.KG, c.cpg_shift, x.D, x.H,
                                                          x.W, x.ld, y.ld, self.rt.code)

    def fwd(self, x: Act, y: Act, stats_part: Optional[torch.Tensor] = None):
        c, L = self.c0, self.rt.lib
        M, nc = x.N * x.V, c.ncols_f
        if stats_part is not None:
            with TIMER.region(_gemm_name(self.rt, nc, "conv3"), flops=2.0 * M * c.Co * 27 * c.Ci,
                              nbytes=_io_bytes(self.rt, M, c.Cip, c.Co, self.G * 27 * c.Cip * c.Co)):
                L.mmseg_conv_gemm_group_stats(x.ptr, x.ld, ptr(c.wf), ptr(c.conv.bias), y.ptr, y.ld, MODE_CONV3, M, nc,
                                              c.Cpad, c.KG, c.cpg_shift, x.D, x.H, x.W, c.kreal_f, self.G, self.w_gs,
                                              self.b_gs, ptr(stats_part), self.rt.code, self.rt.stream)
            return
        ks = L.mmseg_conv3_group_splits(M, nc, c.Cpad, c.KG, c.cpg_shift, x.D, x.H, x.W, x.ld, y.ld, self.rt.code)
        ws = self.rt.ws(ks * M * nc) if ks > 1 else None
        with TIMER.region(_gemm_name(self.rt, nc, "conv3"), flops=2.0 * M * c.Co * 27 * c.Ci,
                          nbytes=_io_bytes(self.rt, M, c.Cip, c.Co, self.G * 27 * c.Cip * c.Co)):
            L.mmseg_conv_gemm_group(x.ptr, x.ld, ptr(c.wf), ptr(c.conv.bias), y.ptr, y.ld, ptr(ws), MODE_CONV3, M, nc,
                                    c.Cpad, c.KG, c.cpg_shift, x.D, x.H, x.W, ks, c.kreal_f, self.G, self.w_gs,
                                    self.b_gs, self.rt.code, self.rt.stream)

    def bwd(self, x: Act, dy: Act, dx: Optional[Act], accumulate: bool):
        """Weight / bias gradients of every group (one weight-gradient launch, one reduce -- on the side stream
        beside the data gradient, as Conv3.bwd), then the data gradient dx (one launch)."""
        c, L, code = self.c0, self.rt.lib, self.rt.code
        V = x.N * x.V
        wsf = L.mmseg_conv3_wgrad_group_ws_floats(V, c.Co, c.Cip, c.Ci, c.cpg_shift, x.D, x.H, x.W, dy.ld, x.ld,
                                                  self.G, code)
        defer = wsf > 0 and self.rt.defer_wred(self.flat)
        ws = c._part(wsf, own=defer)
        gw = ptr(self.flat.grad(c.conv.weight))
        gb = ptr(self.flat.grad(c.conv.bias)) if c.conv.bias is not None else None
        args = (dy.ptr, dy.ld, x.ptr, x.ld, gw, gb, c.Co, c.Cip, c.Ci, c.cpg_shift, V, x.D, x.H, x.W, ptr(ws), wsf,
                int(accumulate), self.G, self.gw_gs, self.gb_gs)
        def wkernel(s1):
            with TIMER.region(_gemm_name(self.rt, 0, "conv3"), flops=2.0 * V * c.Co * 27 * c.Ci,
                              nbytes=_io_bytes(self.rt, V, c.Cip, c.Co, self.G * 27 * c.Cip * c.Co, 4)):
                L.mmseg_conv3_wgrad_group(*args, 1, code, s1)

        def reduce(s2):
            with TIMER.region("wgrad_reduce_kernel"):
                L.mmseg_conv3_wgrad_group(*args, 6 if defer else 2, code, s2)
            for cc in self.convs:
                self.flat.mark(*[p for p in (cc.conv.weight, cc.conv.bias) if p is not None])
        wkernel(self.rt.stream)
        c._reduce_after(reduce)
        try:
            if dx is None:
                return
            M, nc = V, c.ncols_d
            ks = L.mmseg_conv3_group_splits(M, nc, c.Cpad_d, c.KGd, c.dshift, x.D, x.H, x.W, dy.ld, dx.ld, code)
            ws2 = self.rt.ws(ks * M * nc) if ks > 1 else None
            with TIMER.region(_gemm_name(self.rt, nc, "conv3"), flops=2.0 * M * c.Co * 27 * c.Ci,
                              nbytes=_io_bytes(self.rt, M, c.Co, c.Cip, self.G * 27 * c.Cip * c.Co)):
                L.mmseg_conv_gemm_group(dy.ptr, dy.ld, ptr(c.wd), None, dx.ptr, dx.ld, ptr(ws2), MODE_CONV3, M, nc,
                                        c.Cpad_d, c.KGd, c.dshift, x.D, x.H, x.W, ks, c.kreal_d, self.G, self.wd_gs, 0,
                                        code, self.rt.stream)
        finally:
            self.rt.join_side()


def act_group_view(a: Act, g: int, n: int) -> Act:
    """Samples [g n, (g + 1) n) of a combined activation as an Act of its own: a view of the same memory whose
    buffer starts at the group's first sample (Act.off stays the offset inside a voxel row)."""
    span = n * a.V * a.ld
    return Act(a.buf[g * span:(g + 1) * span], a.off, a.C, a.ld, n, a.D, a.H, a.W)


class GroupBlock(Block):
    """The M modality encoders' ConvBlock3D of one small level as one block over M x N samples (ConvGroup convs,
    one-launch InstanceNorm over all M x N samples).  The per-modality Block objects keep views of the combined
    activations and statistics (x1 / y1 / x2 / stats), so everything that reads a modality's block still does."""

    def __init__(self, blocks: List[Block]):
        self.rt = blocks[0].rt
        self.blocks = list(blocks)
        self.G = len(blocks)
        self.g1 = ConvGroup([b.c1 for b in blocks])
        self.g2 = ConvGroup([b.c2 for b in blocks])
        self.c1, self.c2 = blocks[0].c1, blocks[0].c2
        self.Co = blocks[0].Co
        self.shape = None
        self.defer_out = False
        self.defer1 = False
        self.norm1_ok = False

    def setup(self, N, D, H, W):
        """N: samples per modality."""
        if self.shape == (N, D, H, W):
            return
        self.shape = (N, D, H, W)
        rt, C, G = self.rt, self.Co, self.G
        self.x1 = rt.act(G * N, D, H, W, C)
        self.y1 = rt.act(G * N, D, H, W, C)
        self.x2 = rt.act(G * N, D, H, W, C)
        self.stats = torch.empty(4, G * N * C, dtype=torch.float32, device=rt.device)
        self.gnb = None   # fused-statistics bricks per sample of (g1, g2), set on the first forward
        for g, b in enumerate(self.blocks):
            b.shape = (N, D, H, W)
            b.x1, b.y1, b.x2 = (act_group_view(t, g, N) for t in (self.x1, self.y1, self.x2))
            b.stats = self.stats[:, g * N * C:(g + 1) * N * C]
            b.nb, b.norm1_ok, b.defer1, b.defer_out = (0, 0), False, False, False

    def ok(self, xin: Act) -> bool:
        # levels above the one-launch InstanceNorm size group with MMSEG_GROUP_FORCE_R (default on: the 24^3 / 48^3
        # levels on the runtime-brick kernels; the InstanceNorm passes take the multi-pass path over M x N samples)
        small = self.x1.V <= SMALL_IN_V or os.environ.get("MMSEG_GROUP_FORCE_R", "1") != "0"
        return self.g1.ok(xin, self.x1) and self.g2.ok(self.x1, self.x2) and small

    def fwd(self, xin: Act, out: Act):
        st = self.stats
        if self.gnb is None:
            # the statistics from the conv epilogue above the one-launch InstanceNorm size (48^3 / 24^3 with forced
            # grouping); the register-resident small form needs no statistics pass to replace
            big = self.x1.V > SMALL_IN_V
            self.gnb = (self.g1.stats_bricks(xin, self.x1) if big else 0,
                        self.g2.stats_bricks(self.y1, self.x2) if big else 0)
            n = max(self.gnb)
            self.gpart = (torch.empty(self.x1.N * n * self.Co * 2, dtype=torch.float32, device=self.rt.device)
                          if n else None)
        p1 = self.gpart if self.gnb[0] else None
        p2 = self.gpart if self.gnb[1] else None
        self.g1.fwd(xin, self.x1, stats_part=p1)
        self._norm_fwd(self.x1, self.y1, st[0], st[1], p1, self.gnb[0])
        self.g2.fwd(self.y1, self.x2, stats_part=p2)
        self._norm_fwd(self.x2, out, st[2], st[3], p2, self.gnb[1])

    def bwd(self, xin: Act, dy: DySpec, dxin: Optional[Act], accumulate: bool):
        st = self.stats
        g2 = self.x2
        self._norm_bwd(self.x2, st[2], st[3], dy, g2)
        dy1 = self.y1                     # the weight gradient reads y1 before the data gradient overwrites it
        self.g2.bwd(self.y1, g2, dy1, accumulate)
        g1 = self.x1
        self._norm_bwd(self.x1, st[0], st[1], DySpec(p1=dy1), g1)
        self.g1.bwd(xin, g1, dxin, accumulate)


class Head:
    """Dropout3d (per-(n,c) scale) + 1x1 out_conv -> NCDHW fp32 logits."""

    def __init__(self, rt: Runtime, conv: nn.Conv3d, flat: FlatParams):
        self.rt, self.conv, self.flat = rt, conv, flat
        self.C, self.Cin = conv.weight.shape[:2]

    def fwd(self, x: Act, logits: torch.Tensor, dscale: Optional[torch.Tensor]):
        self.dscale = dscale
        self.rt.lib.mmseg_head_fwd(x.ptr, x.ld, self.Cin, ptr(self.conv.weight), ptr(self.conv.bias), ptr(dscale),
                                   self.C, x.N, x.V, ptr(logits), self.rt.code, self.rt.stream)

    # ---- fused head + loss (the Trainer's training step; csrc/loss_head.hip head_loss_*)
    def loss_ok(self, x: Act) -> bool:
        return x.off == 0 and bool(self.rt.lib.mmseg_head_loss_ok(self.C, self.Cin, x.ld, self.rt.code))

    def fwd_loss(self, x: Act, labels: torch.Tensor, spec: dict, cw: Optional[torch.Tensor],
                 dscale: Optional[torch.Tensor], norm: Optional[Tuple[torch.Tensor, torch.Tensor]] = None
                 ) -> torch.Tensor:
        """Head + loss statistics + finalize: the loss scalar, no logits written.  norm = (mean, rstd): x is the
        last decoder block's pre-norm x2 and its InstanceNorm + ReLU is applied on load (Block.defer_out)."""
        L = self.rt.lib
        ws = torch.empty(L.mmseg_loss_ws_floats(x.N, self.C, x.V), dtype=torch.float32, device=self.rt.device)
        loss = torch.empty((), dtype=torch.float32, device=self.rt.device)
        args = (spec["type"], spec["dice_w"], spec["ce_w"], spec["smooth"], spec["alpha"], spec["beta"],
                int(spec["include_bg"]), ptr(cw))
        nm, nr = (ptr(norm[0]), ptr(norm[1])) if norm is not None else (None, None)
        L.mmseg_head_loss_fwd(x.ptr, x.ld, self.Cin, nm, nr, ptr(self.conv.weight), ptr(self.conv.bias), ptr(dscale),
                              self.C, x.N, x.V, ptr(labels), labels.element_size(), *args, ptr(loss), ptr(ws),
                              self.rt.code, self.rt.stream)
        self.loss_state = (labels, args, ws, cw, dscale, (nm, nr))
        return loss, ws

    def in_chunks(self, x: Act) -> int:
        """Chunks per sample of the InstanceNorm-backward partials bwd_loss can emit for the block feeding the head
        (0: not available for this shape or with a Dropout3d scale, or switched off with MMSEG_HEAD_IN_PART=0).
        Call between fwd_loss and bwd_loss."""
        if os.environ.get("MMSEG_HEAD_IN_PART", "1") == "0" or self.loss_state[4] is not None:   # Dropout3d scale
            return 0
        return int(self.rt.lib.mmseg_head_loss_in_chunks(self.C, self.Cin, x.V))

    def bwd_loss(self, x: Act, gout: torch.Tensor, dx: Optional[Act], accumulate: bool,
                 inpart: Optional[torch.Tensor] = None):
        """dlogits (recomputed) -> head data + weight gradient, after fwd_loss.  inpart: also write the
        InstanceNorm-backward partial sums of the head's input block ([N][in_chunks()][Cin][2])."""
        L = self.rt.lib
        labels, args, ws, cw, dscale, (nm, nr) = self.loss_state
        wpart = self.rt.ws(L.mmseg_head_loss_wpart_floats(self.C, self.Cin, x.N, x.V))
        L.mmseg_head_loss_bwd_in(x.ptr, x.ld, self.Cin, nm, nr, ptr(self.conv.weight), ptr(self.conv.bias),
                                 ptr(dscale), self.C, x.N, x.V, ptr(labels), labels.element_size(), *args, ptr(gout),
                                 1.0, ptr(ws), dx.ptr if dx is not None else None, dx.ld if dx is not None else 0,
                                 ptr(self.flat.grad(self.conv.weight)), ptr(self.flat.grad(self.conv.bias)),
                                 ptr(wpart), ptr(inpart), int(accumulate), self.rt.code, self.rt.stream)
        self.flat.mark(self.conv.weight, self.conv.bias)
        self.loss_state = None

    def bwd(self, x: Act, dlogits: torch.Tensor, dx: Optional[Act], accumulate: bool):
        L = self.rt.lib
        ws = self.rt.ws(L.mmseg_head_ws_floats(self.C, self.Cin, x.N, x.V))
        L.mmseg_head_bwd_zw(x.ptr, x.ld, self.Cin, ptr(self.conv.weight), ptr(self.dscale), self.C, x.N, x.V,
                            ptr(dlogits), dx.ptr if dx is not None else None, dx.ld if dx is not None else 0,
                            dx.wcols if dx is not None else self.Cin, ptr(self.flat.grad(self.conv.weight)),
                            ptr(self.flat.grad(self.conv.bias)), ptr(ws), int(accumulate), self.rt.code,
                            self.rt.stream)
        self.flat.mark(self.conv.weight, self.conv.bias)
