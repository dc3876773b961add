"""AdamW over the engine's flat parameter arena: one HIP kernel per step
(mmseg_adamw) instead of torch's per-parameter loop.  Subclasses
torch.optim.AdamW so param_groups / state_dict() / load_state_dict() keep the
torch format the reference's checkpoints use (trainer.py:115-117,
build.py:170-180): per-parameter state 'step', 'exp_avg', 'exp_avg_sq', where
exp_avg / exp_avg_sq are views of two flat fp32 moment buffers."""
from __future__ import annotations

import weakref
from typing import List, Optional

import torch

from .._lib import lib, ptr, stream_handle


def _arena_of(params: List[torch.Tensor]):
    """(base tensor, numel) if the params are consecutive views of one fp32 buffer, else None."""
    p0 = params[0]
    if p0.device.type != "cuda" or any(p.dtype != torch.float32 for p in params):
        return None
    base = p0.data.data_ptr()
    off = 0
    for p in params:
        if p.data.data_ptr() != base + off * 4 or not p.data.is_contiguous():
            return None
        off += p.numel()
    return base, off


def pack_source(model: torch.nn.Module):
    """For FlatAdamW._pack_source: () -> (layers.Packer, FlatParams) of the HIP engine bound to `model` (weakly
    referenced), or None before its first forward."""
    ref = weakref.ref(model)

    def src():
        mdl = ref()
        if mdl is None:
            return None
        bb = getattr(mdl, "backbone", mdl)
        eng = bb.__dict__.get("_engine")
        prog = getattr(eng, "program", None)
        if prog is None or getattr(eng, "flat", None) is None or not hasattr(prog, "packer"):
            return None
        return prog.packer(), eng.flat
    return src


class FlatAdamW(torch.optim.AdamW):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, **kw):
        super().__init__(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, foreach=False, **kw)
        self._flat = {}
        # guard: optional 1-element device tensor (the step's out-of-range label count, Trainer.train_step);
        # the kernel skips the update when it is non-zero (no host sync)
        self.guard: Optional[torch.Tensor] = None

    def _group_step(self, group) -> torch.Tensor:
        """The group's step counter: ONE CPU scalar tensor shared by every parameter's state['step'] (torch's
        checkpoint format keeps a per-parameter 'step'), updated in place -- no per-parameter allocation per
        step.  A state loaded from a checkpoint holds separate tensors; they are merged here."""
        params = group["params"]
        t = self.state[params[0]].get("step")
        if t is None or any(self.state[p].get("step") is not t for p in params):
            t = torch.tensor(float(t) if t is not None else 0.0)
            for p in params:
                self.state[p]["step"] = t
        return t

    def state_dict(self):
        """torch's format with one 'step' tensor PER PARAMETER.  _group_step shares a single counter across a
        group; torch.optim.AdamW (the reference's optimizer, or hardware.kernels: torch resuming an engine
        checkpoint) would otherwise load that sharing and advance the shared tensor once per parameter per
        step, breaking the bias corrections (reference trainer.py:115-117, build.py:170-180)."""
        sd = super().state_dict()
        sd["state"] = {k: ({**st, "step": st["step"].clone()} if torch.is_tensor(st.get("step")) else st)
                       for k, st in sd["state"].items()}
        return sd

    def undo_step_count(self) -> None:
        """Roll the step counters back by one: the kernel skipped an update (guard), so the bias corrections
        of the next step must not advance."""
        for group in self.param_groups:
            t = self._group_step(group)
            t.fill_(max(float(t) - 1.0, 0.0))

    def _moments(self, gi: int, group, numel: int, device):
        params = group["params"]
        m, v = self._flat.get(gi, (None, None))
        if m is None or m.numel() != numel or m.device != device:
            m = torch.zeros(numel, dtype=torch.float32, device=device)
            v = torch.zeros(numel, dtype=torch.float32, device=device)
            self._flat[gi] = (m, v)
        off = 0
        for p in params:
            st = self.state[p]
            n = p.numel()
            mv, vv = m[off:off + n].view_as(p), v[off:off + n].view_as(p)
            if "exp_avg" in st and st["exp_avg"].data_ptr() != mv.data_ptr():
                mv.copy_(st["exp_avg"])      # state loaded from a checkpoint: move into the arena
                vv.copy_(st["exp_avg_sq"])
            st["exp_avg"], st["exp_avg_sq"] = mv, vv
            off += n
        return m, v

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        for gi, group in enumerate(self.param_groups):
            params = [p for p in group["params"]]
            if any(p.grad is None for p in params):
                raise RuntimeError("FlatAdamW: every parameter needs a gradient (engine writes all of them)")
            arena = _arena_of(params)
            garena = _arena_of([p.grad for p in params])
            if arena is None or garena is None:
                raise RuntimeError("FlatAdamW needs the engine's flat parameter/gradient arena on a ROCm device "
                                   "(run one forward/backward through the model first); there is no CPU path")
            if group.get("amsgrad") or group.get("maximize"):
                raise NotImplementedError("FlatAdamW: amsgrad / maximize are not on the HIP path")
            base, n = arena
            m, v = self._moments(gi, group, n, params[0].device)
            st = self._group_step(group)
            step = int(st.item()) + 1
            st.fill_(float(step))
            b1, b2 = group["betas"]
            hyper = (float(group["lr"]), float(b1), float(b2), float(group["eps"]), float(group["weight_decay"]), step)
            # the engine's weight images updated in the same launch (mmseg_adamw_pack) when this arena is the
            # engine's and the images were current, so the next forward skips its pack
            src = self.__dict__.get("_pack_source")
            fp = src() if src is not None and len(self.param_groups) == 1 else None
            pk = tab = None
            if fp is not None and fp[1].flat.data_ptr() == base and fp[1].numel == n:
                pk, flat = fp
                v0 = flat.version()
                tab = pk.adam(flat) if pk.fresh == v0 else None
            if tab is not None:
                lib().mmseg_adamw_pack(base, garena[0], ptr(m), ptr(v), ptr(tab[0]), tab[1], tab[2], *hyper,
                                       ptr(self.guard), pk.rt.code, stream_handle())
            else:
                lib().mmseg_adamw(base, garena[0], ptr(m), ptr(v), n, *hyper, ptr(self.guard), stream_handle())
            # the kernel wrote the weights behind torch's in-place counters: bump them, as torch's AdamW would
            torch.autograd.graph.increment_version(params)
            if tab is not None:
                pk.fresh = flat.version()
        return loss
