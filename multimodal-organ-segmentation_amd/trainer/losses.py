"""Segmentation losses on the MI355X engine — mirror of the reference's
src/trainer/losses.py (DiceLoss 12-80, TverskyLoss 128-185, DiceCELoss
188-228, get_loss 231-267).

Every loss runs as two HIP passes (mmseg_loss_fwd / mmseg_loss_bwd): one pass
computes softmax over C, the one-hot per-(b,c) sums Σp, Σp·t, Σt and the CE
sum with wavefront-shuffle reductions and a fixed-order finalize; the backward
pass writes dlogits directly (no autograd graph of ~10 elementwise ops).
"""
from __future__ import annotations

from typing import Any, Dict, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .._lib import lib, ptr, stream_handle

TYPE_DICE, TYPE_TVERSKY, TYPE_FOCAL = 0, 1, 2


class _SegLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, spec, class_w, owner):
        if logits.device.type != "cuda":
            raise RuntimeError("HIP loss kernels need ROCm tensors; there is no CPU path")
        logits = logits.float().contiguous()
        if target.dtype not in (torch.int64, torch.uint8):
            target = target.long()
        target = target.contiguous()
        N, C = logits.shape[:2]
        V = logits.numel() // (N * C)
        if target.numel() != N * V:
            raise ValueError(f"target shape {tuple(target.shape)} does not match logits {tuple(logits.shape)}")
        L = lib()
        ws = torch.empty(L.mmseg_loss_ws_floats(N, C, V), dtype=torch.float32, device=logits.device)
        loss = torch.empty((), dtype=torch.float32, device=logits.device)
        cw = None if class_w is None else class_w.to(logits.device, torch.float32).contiguous()
        args = (N, C, V, spec["type"], spec["dice_w"], spec["ce_w"], spec["smooth"], spec["alpha"], spec["beta"],
                int(spec["include_bg"]), ptr(cw))
        L.mmseg_loss_fwd(ptr(logits), ptr(target), target.element_size(), *args, ptr(loss), ptr(ws), stream_handle())
        owner.__dict__["_last_ws"] = ws       # its last float = count of labels outside [0, C)
        ctx.save_for_backward(logits, target, ws, cw if cw is not None else torch.empty(0))
        ctx.args = args
        ctx.has_cw = cw is not None
        return loss

    @staticmethod
    def backward(ctx, gout):
        logits, target, ws, cw = ctx.saved_tensors
        N, C, V = ctx.args[:3]
        dlogits = torch.empty_like(logits)
        g = gout.float().contiguous()
        lib().mmseg_loss_bwd(ptr(logits), ptr(target), target.element_size(), *ctx.args, ptr(g), 1.0, ptr(dlogits),
                             ptr(ws), stream_handle())
        return dlogits, None, None, None, None


class _HipLoss(nn.Module):
    """Labels outside [0, C) make the reference raise inside F.one_hot / cross_entropy.  The kernels cannot
    raise without a host sync, so such voxels are skipped, counted on the device and turn the loss into NaN;
    `invalid_labels()` (one sync) reads the count of the last call and `check_labels()` raises on it."""

    def _spec(self) -> Dict[str, Any]:
        raise NotImplementedError

    def invalid_labels(self) -> int:
        ws = self.__dict__.get("_last_ws")
        return 0 if ws is None else int(ws[-1].item())   # coef[2NC+1], the workspace's last float

    def check_labels(self) -> None:
        n = self.invalid_labels()
        if n:
            raise RuntimeError(f"{n} target voxels hold a class index outside [0, num_classes) "
                               "(the reference raises in F.one_hot / cross_entropy on such labels)")

    kernels = "hip"

    def torch_forward(self, pred: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError

    def forward(self, pred: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
        if self.kernels == "torch":
            if pred.device.type != "cuda":
                raise RuntimeError("hardware.kernels: torch runs on a ROCm device; there is no CPU path")
            return self.torch_forward(pred, target)
        if getattr(self, "reduction", "mean") != "mean":
            raise NotImplementedError("HIP losses implement reduction='mean' (the reference's default)")
        return _SegLoss.apply(pred, target, self._spec(), getattr(self, "class_weights", None), self)


class DiceLoss(_HipLoss):
    """softmax -> one-hot -> per-(b,c) (2I+s)/(U+s) -> 1 - dice -> mean (reference losses.py:12-80)."""

    def __init__(self, smooth: float = 1.0, reduction: str = "mean", softmax: bool = True,
                 include_background: bool = True):
        super().__init__()
        if not softmax:
            raise NotImplementedError("HIP DiceLoss applies softmax (reference default)")
        self.smooth, self.reduction, self.softmax, self.include_background = smooth, reduction, softmax, include_background

    def _spec(self):
        return dict(type=TYPE_DICE, dice_w=1.0, ce_w=0.0, smooth=self.smooth, alpha=0.0, beta=0.0,
                    include_bg=self.include_background)

    def torch_forward(self, pred, target):
        """reference losses.py:47-80."""
        C = pred.shape[1]
        p = F.softmax(pred, dim=1)
        t = F.one_hot(target.long(), C).permute(0, 4, 1, 2, 3).float()
        if not self.include_background:
            p, t = p[:, 1:], t[:, 1:]
        p, t = p.flatten(2), t.flatten(2)
        dice = (2.0 * (p * t).sum(-1) + self.smooth) / (p.sum(-1) + t.sum(-1) + self.smooth)
        return _reduce(1.0 - dice, self.reduction)


class CrossEntropyLoss(_HipLoss):
    """nn.CrossEntropyLoss(weight) with mean reduction over B*H*W*D (reference losses.py:214)."""

    def __init__(self, weight: Optional[torch.Tensor] = None):
        super().__init__()
        self.class_weights = weight

    def _spec(self):
        return dict(type=TYPE_DICE, dice_w=0.0, ce_w=1.0, smooth=1.0, alpha=0.0, beta=0.0, include_bg=True)

    def torch_forward(self, pred, target):
        w = None if self.class_weights is None else self.class_weights.to(pred.device)
        return F.cross_entropy(pred, target.long(), weight=w)


class TverskyLoss(_HipLoss):
    """(tp+s)/(tp + a*fp + b*fn + s) per (b,c), 1 - T, mean (reference losses.py:128-185)."""

    def __init__(self, alpha: float = 0.5, beta: float = 0.5, smooth: float = 1.0, reduction: str = "mean"):
        super().__init__()
        self.alpha, self.beta, self.smooth, self.reduction = alpha, beta, smooth, reduction

    def _spec(self):
        return dict(type=TYPE_TVERSKY, dice_w=1.0, ce_w=0.0, smooth=self.smooth, alpha=self.alpha, beta=self.beta,
                    include_bg=True)

    def torch_forward(self, pred, target):
        """reference losses.py:160-185."""
        C = pred.shape[1]
        p = F.softmax(pred, dim=1).flatten(2)
        t = F.one_hot(target.long(), C).permute(0, 4, 1, 2, 3).float().flatten(2)
        tp = (p * t).sum(-1)
        fp = (p * (1 - t)).sum(-1)
        fn = ((1 - p) * t).sum(-1)
        tv = (tp + self.smooth) / (tp + self.alpha * fp + self.beta * fn + self.smooth)
        return _reduce(1.0 - tv, self.reduction)


class FocalLoss(_HipLoss):
    """ce_i = CE(pred, target, weight=alpha, reduction='none'), (1 - exp(-ce_i))^gamma * ce_i, mean over voxels
    (reference losses.py:83-125); gamma rides in the kernel's alpha slot (loss type 2)."""

    def __init__(self, alpha: Optional[torch.Tensor] = None, gamma: float = 2.0, reduction: str = "mean"):
        super().__init__()
        self.alpha, self.gamma, self.reduction = alpha, gamma, reduction
        self.class_weights = alpha

    def _spec(self):
        return dict(type=TYPE_FOCAL, dice_w=0.0, ce_w=1.0, smooth=1.0, alpha=float(self.gamma), beta=0.0,
                    include_bg=True)

    def torch_forward(self, pred, target):
        """reference losses.py:109-125."""
        w = None if self.alpha is None else self.alpha.to(pred.device)
        ce = F.cross_entropy(pred, target.long(), weight=w, reduction="none")
        return _reduce((1 - torch.exp(-ce)) ** self.gamma * ce, self.reduction)


class DiceCELoss(_HipLoss):
    """dice_weight * DiceLoss + ce_weight * CrossEntropy, fused (reference losses.py:188-228)."""

    def __init__(self, dice_weight: float = 0.5, ce_weight: float = 0.5, class_weights: Optional[torch.Tensor] = None,
                 include_background: bool = True):
        super().__init__()
        self.dice_weight, self.ce_weight = dice_weight, ce_weight
        self.class_weights = class_weights
        self.include_background = include_background

    def _spec(self):
        return dict(type=TYPE_DICE, dice_w=self.dice_weight, ce_w=self.ce_weight, smooth=1.0, alpha=0.0, beta=0.0,
                    include_bg=self.include_background)

    def torch_forward(self, pred, target):
        """reference losses.py:216-228."""
        dice = DiceLoss(include_background=self.include_background).torch_forward(pred, target)
        w = None if self.class_weights is None else self.class_weights.to(pred.device)
        return self.dice_weight * dice + self.ce_weight * F.cross_entropy(pred, target.long(), weight=w)


def _reduce(x: torch.Tensor, reduction: str) -> torch.Tensor:
    if reduction == "mean":
        return x.mean()
    if reduction == "sum":
        return x.sum()
    return x


def get_loss(config: Dict[str, Any]) -> nn.Module:
    """reference losses.py:231-267 (+ the hardware.kernels backend, models/build.py)."""
    from ..models.build import kernels_from_config
    loss = _get_loss(config)
    loss.kernels = kernels_from_config(config)
    return loss


def _get_loss(config: Dict[str, Any]) -> nn.Module:
    lc = config["training"]["loss"]
    name = lc["name"].lower()
    cw = lc.get("class_weights")
    cw = torch.tensor(cw, dtype=torch.float32) if cw is not None else None
    if name == "dice":
        return DiceLoss()
    if name in ("ce", "cross_entropy"):
        return CrossEntropyLoss(weight=cw)
    if name == "dice_ce":
        return DiceCELoss(dice_weight=lc.get("dice_weight", 0.5), ce_weight=lc.get("ce_weight", 0.5), class_weights=cw)
    if name == "focal":
        return FocalLoss(alpha=cw)
    if name == "tversky":
        return TverskyLoss(alpha=lc.get("tversky_alpha", 0.5), beta=lc.get("tversky_beta", 0.5))
    return DiceCELoss()
