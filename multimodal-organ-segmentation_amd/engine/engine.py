"""SegEngine: binds a UNet3D / DualEncoder module (the reference's parameter
containers) to its HIP program, and exposes it to torch autograd as ONE
Function: forward runs the whole-network kernel sequence, backward runs the
whole reverse sequence and writes every parameter gradient straight into the
flat gradient arena (p.grad are views of it)."""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn

from .programs import DualEncoderProgram, UNetProgram
from .runtime import FlatParams, Runtime


class SegEngine:
    def __init__(self, module: nn.Module, kind: str):
        self.module = module
        self.kind = kind
        self.rt: Optional[Runtime] = None
        self.flat: Optional[FlatParams] = None
        self.program = None

    def __deepcopy__(self, memo):
        return None  # a copied module builds its own engine / arena on first use

    @property
    def dtype(self) -> torch.dtype:
        return getattr(self.module, "engine_dtype", torch.float32)

    def ensure(self, device: torch.device):
        params = list(self.module.parameters())
        if any(p.device != device for p in params):
            raise RuntimeError(f"model parameters are not on {device}; call model.to({device}) first")
        fp8 = bool(getattr(self.module, "fp8_convs", False))
        if (self.rt is None or self.rt.device != device or self.rt.dtype != self.dtype or self.rt.fp8 != fp8
                or self.flat is None or not self.flat.intact()):
            self.rt = Runtime(device, self.dtype, fp8)
            self.flat = FlatParams(params)
            if self.kind == "swin_unetr":
                from .swin import SwinUNETRProgram
                cls = SwinUNETRProgram
            else:
                cls = UNetProgram if self.kind == "unet" else DualEncoderProgram
            self.program = cls(self.rt, self.module, self.flat)
        return self

    def forward(self, x: torch.Tensor, training: bool) -> torch.Tensor:
        if x.dtype != torch.float32:
            x = x.float()
        x = x.contiguous()
        self.ensure(x.device)
        return self.program.forward(x, training)

    def backward(self, dlogits: torch.Tensor) -> None:
        accumulate = self.flat.begin_backward()
        with self.rt.wred_session():
            self.program.backward(dlogits.float().contiguous(), accumulate)
        self.rt.join_side()
        self.flat.end_backward()

    # ---- fused head + loss (Trainer fast path)
    def forward_loss(self, x: torch.Tensor, training: bool, labels: torch.Tensor, spec: dict,
                     cw: Optional[torch.Tensor]) -> torch.Tensor:
        if x.dtype != torch.float32:
            x = x.float()
        x = x.contiguous()
        self.ensure(x.device)
        loss, ws = self.program.forward(x, training, loss=(labels, spec, cw))
        self.loss_ws = ws
        return loss

    def backward_loss(self, gout: torch.Tensor) -> None:
        accumulate = self.flat.begin_backward()
        with self.rt.wred_session():
            self.program.backward(None, accumulate, gout=gout.float().contiguous())
        self.rt.join_side()
        self.flat.end_backward()


class _EngineFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, anchor, engine, training):
        ctx.engine = engine
        return engine.forward(x, training)

    @staticmethod
    def backward(ctx, dlogits):
        ctx.engine.backward(dlogits)
        # parameter gradients were written by the engine into the flat arena
        return None, None, None, None


class _EngineLossFunction(torch.autograd.Function):
    """Network forward + head + loss as one autograd node (its input is the image, its output the loss)."""

    @staticmethod
    def forward(ctx, x, anchor, engine, training, labels, spec, cw):
        ctx.engine = engine
        return engine.forward_loss(x, training, labels, spec, cw)

    @staticmethod
    def backward(ctx, gout):
        ctx.engine.backward_loss(gout)
        return None, None, None, None, None, None, None


def fused_loss_supported(module: nn.Module, kind: str, x: torch.Tensor) -> bool:
    """True when the network ends in the engine's 1x1 head and the fused head + loss kernels cover its shape
    (UNet3D / DualEncoder, Cin 8 or 32, 2..8 classes)."""
    if kind not in ("unet", "dual_encoder") or x.device.type != "cuda":
        return False
    eng = module.__dict__.get("_engine")
    if eng is None:
        eng = SegEngine(module, kind)
        module.__dict__["_engine"] = eng
    eng.ensure(x.device)
    N, _, D, H, W = x.shape
    eng.program.setup(N, D, H, W)
    return eng.program.loss_ok()


def run_engine_loss(module: nn.Module, kind: str, x: torch.Tensor, labels: torch.Tensor, spec: dict,
                    cw: Optional[torch.Tensor]) -> torch.Tensor:
    """forward + loss in one node (requires fused_loss_supported); backward runs the fused head + loss kernels
    and then the network's backward, writing every parameter gradient into the flat arena."""
    eng = module.__dict__["_engine"]
    anchor = next(module.parameters())
    return _EngineLossFunction.apply(x, anchor, eng, module.training, labels, spec, cw)


def run_engine(module: nn.Module, kind: str, x: torch.Tensor) -> torch.Tensor:
    if x.device.type != "cuda":
        raise RuntimeError("the HIP segmentation engine needs the input on a ROCm device; there is no CPU path")
    eng = module.__dict__.get("_engine")
    if eng is None:
        eng = SegEngine(module, kind)
        module.__dict__["_engine"] = eng
    anchor = next(module.parameters())
    if torch.is_grad_enabled() and anchor.requires_grad:
        return _EngineFunction.apply(x, anchor, eng, module.training)
    with torch.no_grad():
        return eng.forward(x, module.training)
