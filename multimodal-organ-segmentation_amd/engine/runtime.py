"""Device runtime of the segmentation engine: activation views, workspace,
flat parameter / gradient arenas.

Design (MI355X-first, not a translation of the reference's module graph):
  * activations are NDHWC views (`Act`) into device buffers planned once per
    input shape and reused every step, so a whole step is a fixed sequence of
    kernel launches on one HIP stream (hipGraph-capturable);
  * all parameters of a model live in ONE flat fp32 buffer and all gradients
    in another (p.data / p.grad are views), so data-parallel all-reduce moves a
    few large buckets and AdamW is a single kernel over the arena;
  * every kernel is called through the C ABI (`_lib.lib()`); there is no
    eager-PyTorch fallback for any op on the path.
"""
from __future__ import annotations

import math
import os
from contextlib import contextmanager
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import torch

from .._lib import DTYPE_CODE, lib, ptr, stream_handle


@dataclass
class Act:
    """NDHWC activation view: element (n, v, c) at buf[(n*V + v)*ld + off + c]."""
    buf: torch.Tensor
    off: int
    C: int
    ld: int
    N: int
    D: int
    H: int
    W: int
    # the view owns its rows' padding [off + C, ld) (a buffer of its own, not a slot of a wider concat): passes that
    # write it may write zeros there so the rows are written whole (SwinUNETR's 48 / 96-channel tensors at pitch 64 /
    # 128; see mmseg_res_apply's Cw).  CONTRACT: the padding of a whole view holds zeros at all times -- every writer
    # either writes zeros there or leaves it alone, never another value -- because consumers read it as real K
    # columns (the zero-padded weight images multiply it) and the fused dx_add epilogue computes dx_pad + 0.
    # tests/test_swin_unetr_gpu.py::test_swin_whole_act_padding_stays_zero checks it after a forward + backward.
    whole: bool = False

    @property
    def wcols(self) -> int:
        """Channels a pass may write: C, or (a view owning its rows) C rounded up to whole 128-B lines of bf16 (64
        channels) within the pitch -- zeros past C, at most C of them (the kernels' one zero store per real 8-channel
        group)."""
        if not self.whole or self.off:
            return self.C
        w = min(self.ld, -(-self.C // 64) * 64)
        return w if w <= 2 * self.C else self.C

    def pad_max_abs(self) -> float:
        """max |value| in the rows' padding [off + C, ld) over the view's N*V rows (0.0 when there is none)."""
        if self.off + self.C >= self.ld:
            return 0.0
        rows = self.buf[: self.N * self.V * self.ld].view(self.N * self.V, self.ld)
        return rows[:, self.off + self.C:].float().abs().max().item()

    @property
    def V(self) -> int:
        return self.D * self.H * self.W

    @property
    def ptr(self) -> int:
        return self.buf.data_ptr() + self.off * self.buf.element_size()

    def slot(self, off: int, C: int) -> "Act":
        return Act(self.buf, self.off + off, C, self.ld, self.N, self.D, self.H, self.W)

    def to_ncdhw(self) -> torch.Tensor:
        """Debug/test helper: materialise as a float32 NCDHW tensor (a copy)."""
        t = self.buf[: self.N * self.V * self.ld].view(self.N, self.D, self.H, self.W, self.ld)
        return t[..., self.off:self.off + self.C].permute(0, 4, 1, 2, 3).float().contiguous()


class Runtime:
    """Per-model device context: dtype, workspace arena, flat param/grad arenas."""

    def __init__(self, device: torch.device, dtype: torch.dtype, fp8: bool = False):
        if device.type != "cuda":
            raise RuntimeError(
                "the MI355X segmentation engine runs on a ROCm device only (got %s); "
                "there is no CPU fallback" % device)
        if dtype not in DTYPE_CODE:
            raise ValueError(f"engine dtype must be float32 or bfloat16, got {dtype}")
        self.device = device
        self.dtype = dtype
        self.code = DTYPE_CODE[dtype]
        # mixed bf16/fp8 (hardware.fp8, config c5): the forward 3^3 convs that mmseg_conv3_fp8_ok accepts run with
        # e4m3 operands (layers.Conv3); everything else keeps the bf16 storage
        if fp8 and dtype != torch.bfloat16:
            raise ValueError("hardware.fp8 needs hardware.engine_dtype: bfloat16 (the rest of the step stays bf16)")
        self.fp8 = fp8
        self.lib = lib()
        self._ws: Dict[int, torch.Tensor] = {}      # one scratch arena per HIP stream
        # weight-gradient split reduces in line: on a side stream beside the layer's data-gradient kernel they
        # measured +0.3 ms per 96^3 step (6.45 -> 6.75 ms, r04c A/B) -- in the captured graph every fork / join is a
        # cross-queue dependency that costs more than the overlap wins -- and were removed (round 6)
        self.async_wred = False
        self._side: Optional[torch.cuda.Stream] = None
        self._side_pending = False
        # weight-gradient split reduces batched (MMSEG_WRED_BATCH): inside a backward session (`wred_session`) each
        # layer's reduce is queued in the library (its partials in a buffer of the layer's own) and the whole
        # backward's reduces run as one launch at the end of the session -- bitwise the same gradients, 22 fewer
        # launches per 96^3 step (r04h A/B: 6.37 -> 6.31 ms).  Not with DP gradient buckets (they need each
        # gradient as soon as it is final); MMSEG_WRED_BATCH=0 restores one reduce per layer
        self.batch_wred = os.environ.get("MMSEG_WRED_BATCH", "1") != "0"
        self._wred_active = False
        self._wred_session = 0          # id of the current backward session (own_part's reuse check)
        self._wred_flush_hook = None    # DP: flushes the queued reduces before a gradient bucket is reduced

    # ---------------------------------------------------------------- alloc
    def act(self, N: int, D: int, H: int, W: int, C: int, ld: Optional[int] = None) -> Act:
        ld = C if ld is None else ld
        buf = torch.empty(N * D * H * W * ld, dtype=self.dtype, device=self.device)
        return Act(buf, 0, C, ld, N, D, H, W)

    def ws(self, nfloats: int) -> torch.Tensor:
        """Scratch fp32 workspace shared by consecutive ops on the CURRENT stream (each stream has its own,
        so programs that run independent work on side streams never share scratch)."""
        nfloats = int(max(nfloats, 1))
        key = self.stream
        cur = self._ws.get(key)
        if cur is None or cur.numel() < nfloats:
            cur = torch.empty(int(nfloats * 1.25) + 1024, dtype=torch.float32, device=self.device)
            self._ws[key] = cur
        return cur

    @property
    def stream(self) -> int:
        return stream_handle()

    def fork_side(self):
        """Context: the side stream, after everything issued so far on the current stream (a fork of the capture
        stream when a step graph is being captured)."""
        main = torch.cuda.current_stream(self.device)
        if self._side is None:
            self._side = torch.cuda.Stream(self.device)
        self._side.wait_stream(main)
        self._side_pending = True
        return torch.cuda.stream(self._side)

    def defer_wred(self, flat: Optional["FlatParams"]) -> bool:
        """Queue this layer's split reduce until the session ends (see batch_wred).  Under DP gradient buckets the
        queue is flushed before each bucket's collective (FlatParams.flush_before_ready), so the bucketed step
        runs the same batched reduces as the single-GPU one."""
        return (self._wred_active and not self.async_wred
                and (flat is None or flat.on_ready is None or flat.flush_before_ready is not None))

    def own_part(self, obj, nfloats: int) -> torch.Tensor:
        """The split-partial buffer of `obj`'s own for a queued (deferred) reduce.  If obj already queued a reduce
        in this session (a layer whose backward runs twice before the flush), that reduce still has to read the
        buffer: flush the queue first, so the new weight-gradient kernel cannot overwrite partials a queued reduce
        has not summed yet."""
        if getattr(obj, "_wpart_session", None) == self._wred_session and self._wred_active:
            self.flush_wred()
        obj._wpart_session = self._wred_session
        buf = getattr(obj, "_wpart", None)
        if buf is None or buf.numel() < nfloats:
            buf = obj._wpart = torch.empty(int(nfloats), dtype=torch.float32, device=self.device)
        return buf

    def flush_wred(self) -> None:
        """Launch every queued reduce of the current stream now (one batched launch)."""
        n = self.lib.mmseg_wgrad_reduce_flush(self.stream)
        if n < 0:
            raise RuntimeError("mmseg_wgrad_reduce_flush: " + self.lib.mmseg_last_error().decode(errors="replace"))
        # every earlier queued buffer is free again: a layer may defer once more in this session
        self._wred_session += 1

    @contextmanager
    def wred_session(self):
        """A backward whose split reduces may be batched; flushed (one launch) on exit."""
        self._wred_active = self.batch_wred
        self._wred_session += 1
        try:
            yield
        except BaseException:
            self.lib.mmseg_wgrad_reduce_discard(self.stream)
            raise
        finally:
            self._wred_active = False
        if self.batch_wred:
            self.flush_wred()

    def join_side(self) -> None:
        """The current stream waits for all side-stream work (end of the backward: the gradients are final)."""
        if self._side_pending:
            torch.cuda.current_stream(self.device).wait_stream(self._side)
            self._side_pending = False


class FlatParams:
    """Flattens a module's parameters (registration order) into one fp32
    device buffer and their gradients into another; p.data / p.grad become
    views.  Gradients are written by the engine (accumulate flag per step)."""

    def __init__(self, params: List[torch.nn.Parameter]):
        self.params = list(params)
        self.offsets: List[int] = []
        off = 0
        for p in self.params:
            self.offsets.append(off)
            off += p.numel()
        self.numel = off
        dev = self.params[0].device
        self.flat = torch.empty(off, dtype=torch.float32, device=dev)
        self.grad_flat = torch.zeros(off, dtype=torch.float32, device=dev)
        with torch.no_grad():
            for p, o in zip(self.params, self.offsets):
                self.flat[o:o + p.numel()].copy_(p.detach().reshape(-1))
                p.data = self.flat[o:o + p.numel()].view_as(p)
        self.grad_views = [self.grad_flat[o:o + p.numel()].view_as(p) for p, o in zip(self.params, self.offsets)]
        self.index: Dict[int, int] = {id(p): i for i, p in enumerate(self.params)}
        self.sizes = [p.numel() for p in self.params]
        self.on_ready = None      # callback(param_index) once the param's gradient is final (DP buckets)
        # DP with batched weight-gradient reduces: called (by the buckets) right before a bucket's collective is
        # issued, so the reduces still queued in the library have written that bucket's gradients
        self.flush_before_ready = None

    def mark(self, *params: torch.nn.Parameter) -> None:
        if self.on_ready is not None:
            for p in params:
                self.on_ready(self.index[id(p)])

    def version(self) -> Tuple[int, int]:
        """Torch's in-place version counters of the arena and of every parameter: any torch write to the weights
        (load_state_dict, an in-place op on a parameter or on the arena) changes it.  The engine's own kernels
        bypass the counters; FlatAdamW bumps them after its update (torch's AdamW does as much).  The weight packs
        (layers.Packer.fresh) compare against it to skip re-packing unchanged weights."""
        return self.flat._version, sum(p._version for p in self.params)

    def intact(self) -> bool:
        """True if every p.data is still a view of the arena (a .to()/load may rebind it)."""
        base = self.flat.data_ptr()
        es = 4
        return all(p.data.data_ptr() == base + o * es and p.dtype == torch.float32
                   for p, o in zip(self.params, self.offsets))

    def grad(self, p: torch.nn.Parameter) -> torch.Tensor:
        return self.grad_views[self.index[id(p)]]

    def begin_backward(self) -> bool:
        """Returns `accumulate`: False when grads were cleared (p.grad None),
        True when the step accumulates into existing grads (accumulation_steps > 1)."""
        accumulate = all(p.grad is not None for p in self.params)
        if accumulate:
            # re-attach if a user replaced p.grad by a fresh tensor
            for p, g in zip(self.params, self.grad_views):
                if p.grad.data_ptr() != g.data_ptr():
                    g.copy_(p.grad)
        return accumulate

    def end_backward(self) -> None:
        for p, g in zip(self.params, self.grad_views):
            if p.grad is None or p.grad.data_ptr() != g.data_ptr():
                p.grad = g


def pow2_shift(c8: int) -> int:
    s = int(round(math.log2(c8)))
    if (1 << s) != c8:
        raise ValueError(f"channel count {c8 * 8} must be 8 x a power of two")
    return s


def round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m
