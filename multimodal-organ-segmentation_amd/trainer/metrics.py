"""Dice metric on the MI355X engine — mirror of the reference's
DiceMetric (src/trainer/metrics.py:11-88) and get_metrics (229-244).

Counts are integer and exact on the device (mmseg_dice_counts*); each update's
counts are then added into fp32 accumulators exactly as the reference adds its
per-batch fp32 sums, so `compute()` is bit-identical to the reference's on the
same masks.  No per-batch host copy (the reference does .cpu() per update).
"""
from __future__ import annotations

from typing import Any, Dict, Optional

import torch

from .._lib import lib, ptr, stream_handle


class DiceMetric:
    def __init__(self, num_classes: int, include_background: bool = False, reduction: str = "mean",
                 device: Optional[torch.device] = None):
        self.num_classes = num_classes
        self.include_background = include_background
        self.reduction = reduction
        self.device = device       # accumulators live here from the start (a rank with no batches still packs them)
        self.reset()

    def reset(self) -> None:
        self.intersection = torch.zeros(self.num_classes, device=self.device)
        self.union = torch.zeros(self.num_classes, device=self.device)
        self.count = 0
        self._counts: Optional[torch.Tensor] = None

    def _accumulate(self, counts: torch.Tensor) -> None:
        C = self.num_classes
        c = counts.to(torch.float32)
        if self.intersection.device != counts.device:
            self.intersection = self.intersection.to(counts.device)
            self.union = self.union.to(counts.device)
        self.intersection += c[:C]
        self.union += c[C:2 * C] + c[2 * C:]
        self.count += 1

    def _scratch(self, device) -> torch.Tensor:
        if self._counts is None or self._counts.device != device:
            self._counts = torch.zeros(3 * self.num_classes, dtype=torch.int64, device=device)
        else:
            self._counts.zero_()
        return self._counts

    def update(self, pred: torch.Tensor, target: torch.Tensor) -> None:
        """pred / target: class-index masks [B, H, W, D] (reference metrics.py:42-67)."""
        if pred.device.type != "cuda":
            raise RuntimeError("HIP DiceMetric needs ROCm tensors; there is no CPU path")
        pred = pred.contiguous() if pred.dtype in (torch.int64, torch.uint8) else pred.long().contiguous()
        target = target.contiguous() if target.dtype in (torch.int64, torch.uint8) else target.long().contiguous()
        counts = self._scratch(pred.device)
        lib().mmseg_dice_counts_idx(ptr(pred), pred.element_size(), ptr(target), target.element_size(), pred.numel(),
                                    self.num_classes, ptr(counts), stream_handle())
        self._accumulate(counts)

    def update_from_logits(self, logits: torch.Tensor, target: torch.Tensor) -> None:
        """Fused argmax(dim=1) + update (trainer.py:290-291) without materialising the mask."""
        logits = logits.float().contiguous()
        target = target.contiguous() if target.dtype in (torch.int64, torch.uint8) else target.long().contiguous()
        N, C = logits.shape[:2]
        V = logits.numel() // (N * C)
        counts = self._scratch(logits.device)
        lib().mmseg_dice_counts(ptr(logits), ptr(target), target.element_size(), N, C, V, ptr(counts), None,
                                stream_handle())
        self._accumulate(counts)

    def compute(self) -> Dict[str, Any]:
        smooth = 1e-5
        dpc = (2.0 * self.intersection.cpu() + smooth) / (self.union.cpu() + smooth)
        start = 0 if self.include_background else 1
        return {"dice": dpc[start:].mean().item(), "dice_per_class": dpc.tolist()}


def get_metrics(config: Dict[str, Any]) -> Dict[str, Any]:
    """reference metrics.py:229-244 (ConfusionMatrix is never used by the reference trainer)."""
    return {"dice": DiceMetric(num_classes=config["model"]["out_channels"])}
