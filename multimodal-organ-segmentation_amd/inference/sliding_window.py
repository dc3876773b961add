"""Sliding-window inference on device — the reference's Trainer._sliding_window_inference
(trainer.py:370-395) calls MONAI's `sliding_window_inference(image, roi_size, sw_batch_size,
predictor, overlap)` with the config's inference block (configs/default.yaml:127-133).  MONAI is
absent from this image, so its published algorithm (MONAI 1.3,
monai/inferers/utils.py sliding_window_inference, monai/data/utils.py dense_patch_slices) is
restated here for the arguments the reference passes: `mode` is not passed, so blending is
"constant" (the YAML's "gaussian" is dead config); padding is zeros.

Window cutting, accumulation and normalisation are HIP kernels (csrc/inference.hip); the
predictor is the engine model.  Windows are accumulated one at a time in MONAI's order, so each
output voxel is the same fp32 sum MONAI forms (parity is checked against the CPU restatement in
oracle/mmseg_oracle.py; against MONAI itself it is unpinned).
"""
from __future__ import annotations

import math
from typing import Callable, List, Sequence, Tuple

import torch

from .._lib import lib, ptr, stream_handle


def window_starts(size: int, roi: int, overlap: float) -> Tuple[List[int], int]:
    """Window starts along one axis in MONAI's padded frame, and the padding before it.
    (_get_scan_interval + dense_patch_slices of MONAI 1.3, one dimension.)"""
    padded = max(size, roi)
    pad_before = (padded - size) // 2
    if roi == padded:
        interval = roi
    else:
        interval = max(int(roi * (1 - overlap)), 1)
    num = int(math.ceil(float(padded) / interval))
    scan = next((d for d in range(num) if d * interval + roi >= padded), None)
    count = scan + 1 if scan is not None else 1
    starts = []
    for i in range(count):
        s = i * interval
        s -= max(s + roi - padded, 0)
        starts.append(s)
    return starts, pad_before


def _coverage(size: int, starts: List[int], pad_before: int, roi: int) -> torch.Tensor:
    c = torch.zeros(size, dtype=torch.float32)
    for s in starts:
        lo, hi = max(s - pad_before, 0), min(s - pad_before + roi, size)
        c[lo:hi] += 1.0
    return c


def sliding_window_inference(inputs: torch.Tensor, roi_size: Sequence[int], sw_batch_size: int,
                             predictor: Callable[[torch.Tensor], torch.Tensor], overlap: float = 0.25) -> torch.Tensor:
    """inputs [N, M, D, H, W] fp32 on the device -> [N, C, D, H, W] fp32 (MONAI semantics, constant blending)."""
    if inputs.dim() != 5 or inputs.device.type != "cuda":
        raise RuntimeError("sliding_window_inference runs on the ROCm device, input [N, M, D, H, W]")
    if not 0 <= overlap < 1:
        raise ValueError("overlap must be >= 0 and < 1")
    x = inputs.float().contiguous()
    N, M, D, H, W = x.shape
    dims = (D, H, W)
    roi = [r if r > 0 else s for r, s in zip(roi_size, dims)]     # fall_back_tuple
    axes = [window_starts(s, r, overlap) for s, r in zip(dims, roi)]
    wins = []
    for n in range(N):                          # MONAI: windows image-major, then meshgrid "ij" order
        for z in axes[0][0]:
            for y in axes[1][0]:
                for xx in axes[2][0]:
                    wins.append((n, z - axes[0][1], y - axes[1][1], xx - axes[2][1]))
    L, s = lib(), stream_handle()
    dev = x.device
    win_dev = torch.tensor(wins, dtype=torch.int32).reshape(-1).to(dev)
    out = None
    C = None
    rv = roi[0] * roi[1] * roi[2]
    for b0 in range(0, len(wins), sw_batch_size):
        nb = min(sw_batch_size, len(wins) - b0)
        batch = torch.empty(nb, M, *roi, dtype=torch.float32, device=dev)
        L.mmseg_window_gather(ptr(x), N, M, D, H, W, ptr(win_dev) + 16 * b0, nb, roi[0], roi[1], roi[2], ptr(batch), s)
        logits = predictor(batch)
        if isinstance(logits, (tuple, list)):
            logits = logits[0]
        logits = logits.float().contiguous()
        if out is None:
            C = logits.shape[1]
            out = torch.zeros(N, C, D, H, W, dtype=torch.float32, device=dev)
        for k in range(nb):
            n, z0, y0, x0 = wins[b0 + k]
            L.mmseg_window_accum(ptr(logits) + 4 * k * C * rv, N, C, D, H, W, n, z0, y0, x0, roi[0], roi[1], roi[2],
                                 ptr(out), s)
    cov = [_coverage(sz, st, pb, r).to(dev) for sz, (st, pb), r in zip(dims, axes, roi)]
    L.mmseg_window_norm(ptr(out), N, C, D, H, W, ptr(cov[0]), ptr(cov[1]), ptr(cov[2]), s)
    return out
