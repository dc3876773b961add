"""The training step as a captured HIP graph (reference trainer.py:250-258: forward, loss, backward, optimizer
step -- accumulation 1).

Submitting one eager step costs ~4.3 ms of host time for ~300 launches through ctypes (DESIGN (d) "Host"), about
as long as the GPU takes for the whole 96^3 step, so below that the step is bound by Python, not by the kernels.
Every launch of the step goes through the enqueue-only C ABI on the current stream with buffers planned once
per input shape, so the step is capturable as it stands: forward + fused head / loss (engine.forward_loss),
backward (program.backward with a constant output gradient of 1) and the AdamW kernel are captured once per input
(address, shape) and replayed with one host call.

What changes per step lives in device memory, not in kernel arguments:
  * the AdamW hyper-parameters (lr from the scheduler, the bias corrections of step t) -- mmseg_adamw_dev reads
    8 floats that mmseg_adamw_hyper fills on the host; they go through a ring of pinned buffers (an event per
    slot guards reuse) and one async copy before each replay;
  * the inputs: a graph reads the images / labels at the addresses it was captured with, so graphs are cached
    per (address, shape, dtype) of the batch (the pre-staged batches of a benchmark, or the few addresses a
    caching allocator cycles through); past MAX_GRAPHS distinct inputs the batch is copied into the static
    input buffers of one more graph.
The replayed step runs the same kernels in the same order on the same buffers as the eager step, so it is
bitwise equal to it (tests/test_step_graph_gpu.py).

Data parallel over RCCL: the bucket all-reduces (ddp.GradBuckets, issued from the engine's gradient-ready
callbacks) are recorded into the same graph at the points of the backward where they were issued, on the comm
stream forked from the capture stream, so the replayed DP step overlaps them with the rest of the backward
exactly as the eager step does, without ~4 ms of host submission per step.  gloo (host-side collectives) stays
eager.

Used when the step has nothing per-step on the host side: accumulation_steps 1, the engine's fused head + loss, FlatAdamW (one group, no amsgrad),
no Dropout3d in training, single-stream engine, kernel timer off, optimizer.step / zero_grad not wrapped by the
caller (a replay does not call them).  hardware.step_graph: false or MMSEG_STEP_GRAPH=0 turns it off.
"""
from __future__ import annotations

import gc
import os
import weakref
from collections import OrderedDict
from typing import Optional, Tuple

import torch

from .._lib import lib, ptr, stream_handle


class StepGraphs:
    MAX_GRAPHS = 4       # pointer-keyed graphs (the bench pre-stages 4 batches)
    RING = 16            # pinned hyper-parameter slots

    def __init__(self, trainer):
        # a weak reference: no Trainer <-> StepGraphs cycle, so a dropped Trainer frees its graphs at once (by
        # reference count) instead of whenever the cyclic collector runs -- which may be in the middle of another
        # trainer's capture, where destroying a graph is an error (hipErrorStreamCaptureUnsupported)
        self._tr = weakref.ref(trainer)
        self.graphs: "OrderedDict[tuple, dict]" = OrderedDict()
        self.copy_graph: Optional[dict] = None
        self.dev = trainer.device
        self.gout = torch.ones((), dtype=torch.float32, device=self.dev)
        self.hyper_dev = torch.zeros(8, dtype=torch.float32, device=self.dev)
        self.ring = [torch.zeros(8, dtype=torch.float32).pin_memory() for _ in range(self.RING)]
        self.ring_ev = [None] * self.RING
        self.slot = 0

    @property
    def tr(self):
        return self._tr()

    # ------------------------------------------------------------------ eligibility
    def usable(self, images: torch.Tensor, labels: torch.Tensor) -> bool:
        env = os.environ.get("MMSEG_STEP_GRAPH")
        if env == "0" or (env is None and not self.tr.config["hardware"].get("step_graph", True)):
            return False
        from ..engine.profiler import TIMER
        from .optim import FlatAdamW
        tr = self.tr
        if TIMER.enabled or tr.accumulation_steps != 1:
            return False
        if tr.dp:
            # RCCL collectives are capturable (recorded on the comm stream forked from the capture stream); gloo's
            # run on the host and are not.  MMSEG_STEP_GRAPH_DP=0 keeps the DP step eager.
            from ..distributed import ddp
            if ddp.backend() != "nccl" or os.environ.get("MMSEG_STEP_GRAPH_DP", "1") == "0":
                return False
            if ddp.world() > 1 and not getattr(self, "_warned_dp", False):
                # bitwise-tested at world size 1 over RCCL (test_rccl_dp_step_captured_bitwise_equal_to_eager);
                # across several ranks (collectives recorded in each rank's graph, every rank capturing at the same
                # step because all key their graphs on the same batch sequence) it has not run on hardware yet
                import warnings
                warnings.warn("captured data-parallel step over RCCL with world size > 1: verified at world size 1 "
                              "only; MMSEG_STEP_GRAPH_DP=0 keeps the DP step eager", RuntimeWarning, stacklevel=2)
                self._warned_dp = True
        if os.environ.get("MMSEG_MODALITY_STREAMS", "0") != "0":
            return False
        opt = tr.optimizer
        if type(opt) is not FlatAdamW or len(opt.param_groups) != 1:
            return False
        wrapped = opt.__dict__.get("step")
        if (wrapped is not None and not getattr(wrapped, "_wrapped_by_lr_sched", False)) or "zero_grad" in opt.__dict__:
            return False   # a caller wrapped the optimizer's step: a replayed step would not call it
        # (an LR scheduler's wrapper only records that step() ran -- run() sets that flag itself)
        grp = opt.param_groups[0]
        if grp.get("amsgrad") or grp.get("maximize"):
            return False
        bb = getattr(tr.model, "backbone", tr.model)
        if getattr(bb, "dropout_p", 0.0) > 0 and tr.model.training:
            return False
        if not tr.model.training or images.device.type != "cuda" or labels.device.type != "cuda":
            return False
        if images.dtype != torch.float32 or labels.dtype not in (torch.int64, torch.uint8):
            return False
        return images.is_contiguous() and labels.is_contiguous()

    def _engine_key(self):
        """Identity of every buffer a graph bakes in: a rebuilt engine (new arenas / activation plan) or newly
        allocated optimizer moments invalidate the captured graphs."""
        bb = getattr(self.tr.model, "backbone", self.tr.model)
        eng = bb.__dict__.get("_engine")
        if eng is None or eng.flat is None:
            return None
        mv = self.tr.optimizer._flat.get(0, (None, None))
        return (id(eng.program), id(eng.flat), eng.flat.flat.data_ptr(), eng.flat.grad_flat.data_ptr(),
                eng.program.shape, None if mv[0] is None else mv[0].data_ptr(),
                None if mv[1] is None else mv[1].data_ptr())

    # ------------------------------------------------------------------ capture
    def _capture(self, x: torch.Tensor, y: torch.Tensor) -> dict:
        tr = self.tr
        bb = getattr(tr.model, "backbone", tr.model)
        eng = bb.__dict__["_engine"]
        crit = tr.criterion
        spec = crit._spec()
        cw = getattr(crit, "class_weights", None)
        cw = None if cw is None else cw.to(self.dev, torch.float32).contiguous()
        opt = tr.optimizer
        grp = opt.param_groups[0]
        flat = eng.flat
        m, v = opt._moments(0, grp, flat.numel, self.dev)
        L = lib()
        # the fused AdamW + pack launch (mmseg_adamw_pack_dev) keeps the weight images current, so the captured
        # forward leaves out its pack; run() packs eagerly before a replay only when the images are not current
        prog = eng.program
        pk = prog.packer() if hasattr(prog, "packer") else None
        fused = pk.adam(flat) if pk is not None else None
        g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize(self.dev)
        # no cyclic garbage collection while capturing: a collected object owning a graph (or anything that frees
        # device memory through the runtime) would be destroyed inside the capture
        gc_on = gc.isenabled()
        gc.collect()
        gc.disable()
        prog.skip_pack = fused is not None
        try:
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                loss = eng.forward_loss(x, True, y, spec, cw)
                ws = eng.loss_ws
                # DP: the bucket all-reduces are issued by the engine's gradient-ready callbacks during the backward
                # (recorded into the graph on the comm stream), the guard count travels with the first bucket,
                # and finish() joins every collective into the capture stream before the AdamW kernel
                tr._arm_buckets(True, ws[-1:])
                with eng.rt.wred_session():
                    eng.program.backward(None, False, gout=self.gout)
                eng.rt.join_side()
                if tr.dp and tr._buckets is not None:
                    tr._buckets.finish()
                if fused is not None:
                    L.mmseg_adamw_pack_dev(ptr(flat.flat), ptr(flat.grad_flat), ptr(m), ptr(v), ptr(fused[0]),
                                           fused[1], fused[2], ptr(self.hyper_dev), ptr(ws[-1:]), eng.rt.code,
                                           stream_handle())
                else:
                    L.mmseg_adamw_dev(ptr(flat.flat), ptr(flat.grad_flat), ptr(m), ptr(v), flat.numel,
                                      ptr(self.hyper_dev), ptr(ws[-1:]), stream_handle())
        except BaseException:
            # a capture that fails part-way through the backward (e.g. a collective RCCL cannot capture) has
            # already decremented bucket counts and stored works / events: drop them so the eager fallback
            # fires every bucket exactly once
            if tr._buckets is not None:
                tr._buckets.reset()
            raise
        finally:
            prog.skip_pack = False
            if gc_on:
                gc.enable()
        return {"graph": g, "loss": loss, "ws": ws, "x": x, "y": y, "cw": cw, "prog": prog, "packer": pk,
                "fused_pack": fused is not None, "fused_table": fused}

    def _entry(self, images: torch.Tensor, labels: torch.Tensor) -> dict:
        ek = self._engine_key()
        if ek != getattr(self, "_ek", None):
            self.graphs.clear()
            self.copy_graph = None
        key = (images.data_ptr(), tuple(images.shape), labels.data_ptr(), tuple(labels.shape), labels.dtype)
        e = self.graphs.get(key)
        if e is not None and ek == getattr(self, "_ek", None):
            self.graphs.move_to_end(key)
            return e
        if len(self.graphs) < self.MAX_GRAPHS:
            e = self._capture(images, labels)
            self.graphs[key] = e
            self._ek = self._engine_key()
            return e
        # more distinct inputs than pointer-keyed graphs: one graph over static input buffers (+ two D2D copies)
        c = self.copy_graph
        if c is None or c["x"].shape != images.shape or c["y"].shape != labels.shape or c["y"].dtype != labels.dtype:
            sx, sy = torch.empty_like(images), torch.empty_like(labels)
            sx.copy_(images)
            sy.copy_(labels)
            c = self._capture(sx, sy)
            self.copy_graph = c
            self._ek = self._engine_key()
        else:
            c["x"].copy_(images)
            c["y"].copy_(labels)
        return c

    # ------------------------------------------------------------------ replay
    def _push_hyper(self) -> int:
        """Host: next step's AdamW hyper-parameters into a pinned slot, async copy to the device buffer."""
        opt = self.tr.optimizer
        grp = opt.param_groups[0]
        st = opt._group_step(grp)
        step = int(st.item()) + 1
        st.fill_(float(step))
        k = self.slot
        self.slot = (k + 1) % self.RING
        ev = self.ring_ev[k]
        if ev is not None:
            ev.synchronize()          # the copy that last read this slot has run (practically always already)
        b1, b2 = grp["betas"]
        buf = self.ring[k]
        lib().mmseg_adamw_hyper(float(grp["lr"]), float(b1), float(b2), float(grp["eps"]),
                                float(grp["weight_decay"]), step, buf.data_ptr())
        self.hyper_dev.copy_(buf, non_blocking=True)
        if ev is None:
            ev = self.ring_ev[k] = torch.cuda.Event()
        ev.record()
        return step

    def run(self, images: torch.Tensor, labels: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """One training step by graph replay; returns (loss, guard) -- both device tensors owned by the graph (the
        loss is overwritten by the next replay of the same graph)."""
        e = self._entry(images, labels)
        pk = e["packer"]
        if e["fused_pack"]:
            # the captured forward has no pack: the images must be current before the replay (its first one, or
            # weights changed outside the graph since the last); the replay's AdamW + pack keeps them current
            e["prog"].pack()
        self._push_hyper()
        e["graph"].replay()
        if pk is not None and not e["fused_pack"]:
            pk.fresh = None      # the replayed AdamW wrote the weights after the captured pack read them
        # what torch's LRScheduler step wrapper records (lr_scheduler.py patch_track_step_called): the optimizer
        # stepped before the scheduler does, so scheduler.step() raises no "called before optimizer.step()" warning
        self.tr.optimizer.__dict__["_opt_called"] = True
        self.tr.criterion.__dict__["_last_ws"] = e["ws"]
        return e["loss"], e["ws"][-1:]
