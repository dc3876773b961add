"""SwinUNETR entry of the model registry (reference swin_unetr.py:20-200).

The reference wraps monai.networks.nets.SwinUNETR; MONAI is not installed in
this image, so the arithmetic is parity-unpinned.  The MI355X
window-attention implementation is SURVEY §8(f) rank 3 and is not part of
this round's engine: building it raises, exactly like the reference does
when MONAI is missing (swin_unetr.py:71-72).
"""
from __future__ import annotations

from typing import Any, Dict


class SwinUNETR:  # pragma: no cover - not yet on the engine path
    def __init__(self, *args, **kwargs):
        raise ImportError("SwinUNETR is not available on the MI355X engine yet (SURVEY §8f rank 3); "
                          "use model.name 'unet' or 'dual_encoder'")


def build_swin_unetr(config: Dict[str, Any]):
    return SwinUNETR()
