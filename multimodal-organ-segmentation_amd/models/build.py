"""Model factory — mirror of the reference's src/models/build.py
(MODEL_REGISTRY build.py:16-21, build_model 77-114, checkpoints 122-180).

Differences, all additive:
  * `hardware.engine_dtype` ("float32" | "bfloat16") selects the engine's
    activation storage; if absent, `hardware.mixed_precision: true` (the
    reference's fp16-autocast switch) maps to bfloat16 and false to float32.
    Parameters, gradients and optimizer state stay fp32 either way.
  * `hardware.kernels` ("hip" | "torch", default "hip") selects the backend
    (SURVEY §8b): "hip" runs the whole network as one HIP program; "torch"
    runs the same parameter containers through plain PyTorch-ROCm ops (MIOpen
    convolutions), the reference's own module forward, for A/B runs on the
    GPU.  It is chosen explicitly, never as a fallback, and needs a ROCm device
    like the HIP backend.
  * `hardware.fp8: true` (with engine_dtype bfloat16; config c5's "mixed
    bf16/fp8") runs the forward 3^3 convolutions the fp8 kernel takes (one
    32-channel input chunk: the 96^3 conv2 layers) with OCP e4m3 operands and
    fp32 accumulation; backward, norms, fusion and loss stay bf16 / fp32.
"""
from __future__ import annotations

from typing import Any, Dict, Optional

import torch
import torch.nn as nn

from .backbones.dual_encoder import DualEncoder, build_dual_encoder
from .backbones.swin_unetr import SwinUNETR, build_swin_unetr
from .backbones.unet import UNet3D, build_unet3d

MODEL_REGISTRY = {
    "swin_unetr": build_swin_unetr,
    "unet": build_unet3d,
    "unet3d": build_unet3d,
    "dual_encoder": build_dual_encoder,
}


def engine_dtype_from_config(config: Dict[str, Any]) -> torch.dtype:
    hw = config.get("hardware", {})
    name = hw.get("engine_dtype")
    if name is None:
        name = "bfloat16" if hw.get("mixed_precision", False) else "float32"
    table = {"float32": torch.float32, "fp32": torch.float32, "bfloat16": torch.bfloat16, "bf16": torch.bfloat16}
    if name not in table:
        raise ValueError(f"hardware.engine_dtype must be one of {sorted(table)}, got {name!r}")
    return table[name]


KERNELS = ("hip", "torch")


def kernels_from_config(config: Dict[str, Any]) -> str:
    name = str(config.get("hardware", {}).get("kernels", "hip")).lower()
    if name not in KERNELS:
        raise ValueError(f"hardware.kernels must be one of {list(KERNELS)}, got {name!r}")
    return name


class MultiModalSegmentationModel(nn.Module):
    """Pass-through wrapper (reference build.py:24-74): forward(x, return_features)."""

    def __init__(self, backbone: nn.Module, config: Dict[str, Any]):
        super().__init__()
        self.backbone = backbone
        self.config = config
        self.num_modalities = len(config["data"]["modalities"])

    def forward(self, x: torch.Tensor, return_features: bool = False):
        return self.backbone(x, return_features=return_features)

    def load_pretrained(self, path: str) -> None:
        state = torch.load(path, map_location="cpu", weights_only=True)
        if "model_state_dict" in state:
            state = state["model_state_dict"]
        self.load_state_dict(state, strict=False)


def build_model(config: Dict[str, Any]) -> nn.Module:
    name = config["model"]["name"].lower()
    if name not in MODEL_REGISTRY:
        raise ValueError(f"Unknown model: {name}. Available: {list(MODEL_REGISTRY.keys())}")
    n_mod = len(config["data"]["modalities"])
    if name in ("swin_unetr", "unet", "unet3d"):
        config["model"]["in_channels"] = n_mod          # reference build.py:97-99
    kernels = kernels_from_config(config)
    if kernels == "torch" and name == "swin_unetr":
        raise ValueError("hardware.kernels: torch covers unet / dual_encoder, not swin_unetr (MONAI is absent)")
    backbone = MODEL_REGISTRY[name](config)
    backbone.engine_dtype = engine_dtype_from_config(config)
    backbone.kernels = kernels
    # hardware.fp8 (config c5 "mixed bf16/fp8"): e4m3 forward convolutions where the kernels take them
    backbone.fp8_convs = bool(config.get("hardware", {}).get("fp8", False))
    if backbone.fp8_convs and (kernels != "hip" or backbone.engine_dtype != torch.bfloat16):
        raise ValueError("hardware.fp8 needs hardware.kernels: hip and engine_dtype: bfloat16")
    model = MultiModalSegmentationModel(backbone, config)
    if config.get("hardware", {}).get("device", "cuda") == "cuda" and torch.cuda.is_available():
        model = model.cuda()
    return model


def get_model(config: Dict[str, Any]) -> nn.Module:
    return build_model(config)


def load_checkpoint(model: nn.Module, checkpoint_path: str, strict: bool = False) -> Dict[str, Any]:
    """reference build.py:122-150 (safe loader: weights_only=True)."""
    ckpt = torch.load(checkpoint_path, map_location="cpu", weights_only=True)
    if "model_state_dict" in ckpt:
        state = ckpt["model_state_dict"]
    elif "state_dict" in ckpt:
        state = ckpt["state_dict"]
    else:
        state = ckpt
    model.load_state_dict(state, strict=strict)
    return ckpt


def save_checkpoint(model: nn.Module, optimizer: Optional[torch.optim.Optimizer], epoch: int, checkpoint_path: str,
                    **kwargs) -> None:
    """reference build.py:153-180: {epoch, model_state_dict, optimizer_state_dict, **kwargs}."""
    ckpt = {"epoch": epoch, "model_state_dict": model.state_dict()}
    if optimizer is not None:
        ckpt["optimizer_state_dict"] = optimizer.state_dict()
    ckpt.update(kwargs)
    torch.save(ckpt, checkpoint_path)
