"""UNet3D on the MI355X engine — mirror of the reference's
src/models/backbones/unet.py API (class names, constructor arguments,
state-dict names, RNG init order), executed by the HIP engine.

The nn.Modules here are parameter containers: creating them consumes the CPU
RNG in exactly the reference's order (reference unet.py:26-27, 95, 148-163),
so `torch.manual_seed(s); build_model(cfg)` yields bit-identical initial
weights, and reference checkpoints load unchanged.  `UNet3D.forward` runs the
whole network as one HIP program (engine/programs.py); the block modules'
own forward is only the container interface.
"""
from __future__ import annotations

from typing import Any, Dict, List, Tuple, Union

import torch
import torch.nn as nn
import torch.nn.functional as F

from ...engine import run_engine

SUPPORTED_NORM = ("instance",)


class ConvBlock3D(nn.Module):
    """(Conv3d 3^3 pad 1 -> InstanceNorm3d -> ReLU) x 2   (reference unet.py:12-60)."""

    def __init__(self, in_channels: int, out_channels: int, kernel_size: int = 3, padding: int = 1,
                 norm: str = "instance", activation: str = "relu"):
        super().__init__()
        if kernel_size != 3 or padding != 1:
            raise NotImplementedError("engine ConvBlock3D: kernel_size=3, padding=1 only")
        if norm not in SUPPORTED_NORM or activation != "relu":
            raise NotImplementedError(f"engine ConvBlock3D: norm={norm!r}/activation={activation!r} not on the "
                                      "HIP path (reference default instance/relu is)")
        # construction order = RNG order: conv1, conv2, then the parameter-free norms
        self.conv1 = nn.Conv3d(in_channels, out_channels, 3, padding=1)
        self.conv2 = nn.Conv3d(out_channels, out_channels, 3, padding=1)
        self.norm1 = nn.InstanceNorm3d(out_channels)
        self.norm2 = nn.InstanceNorm3d(out_channels)
        self.act = nn.ReLU(inplace=True)

    def forward(self, x):
        """torch-op backend only (reference unet.py:53-60); the HIP backend runs the block inside its program."""
        x = self.act(self.norm1(self.conv1(x)))
        return self.act(self.norm2(self.conv2(x)))


class DownBlock3D(nn.Module):
    """MaxPool3d(2) -> ConvBlock3D   (reference unet.py:63-79)."""

    def __init__(self, in_channels: int, out_channels: int, norm: str = "instance"):
        super().__init__()
        self.pool = nn.MaxPool3d(2)
        self.conv = ConvBlock3D(in_channels, out_channels, norm=norm)

    def forward(self, x):
        """torch-op backend only (reference unet.py:74-79): (conv(pool(x)), pool(x))."""
        x_pool = self.pool(x)
        return self.conv(x_pool), x_pool


class UpBlock3D(nn.Module):
    """ConvTranspose3d(k2,s2) -> cat([up, skip]) -> ConvBlock3D   (reference unet.py:82-113)."""

    def __init__(self, in_channels: int, out_channels: int, norm: str = "instance", mode: str = "transpose"):
        super().__init__()
        if mode != "transpose":
            raise NotImplementedError("engine UpBlock3D: mode='transpose' only (reference default)")
        self.up = nn.ConvTranspose3d(in_channels, in_channels // 2, kernel_size=2, stride=2)
        self.conv = ConvBlock3D(in_channels, out_channels, norm=norm)

    def forward(self, x, skip):
        """torch-op backend only (reference unet.py:104-113)."""
        x = self.up(x)
        if x.shape != skip.shape:
            x = F.interpolate(x, size=skip.shape[2:], mode="trilinear", align_corners=True)
        return self.conv(torch.cat([x, skip], dim=1))


class UNet3D(nn.Module):
    """3D UNet: init block, len(features)-1 down blocks, as many up blocks, 1x1 head
    (reference unet.py:116-205)."""

    def __init__(self, in_channels: int = 1, out_channels: int = 8, features: List[int] = (32, 64, 128, 256, 512),
                 norm: str = "instance", dropout: float = 0.0, **kwargs):
        super().__init__()
        features = [int(f) for f in features]
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.features = features
        self.dropout_p = float(dropout)
        self.init_conv = ConvBlock3D(in_channels, features[0], norm=norm)
        self.encoders = nn.ModuleList(
            [DownBlock3D(a, b, norm=norm) for a, b in zip(features[:-1], features[1:])])
        self.decoders = nn.ModuleList(
            [UpBlock3D(features[i], features[i - 1], norm=norm) for i in range(len(features) - 1, 0, -1)])
        self.dropout = nn.Dropout3d(dropout) if dropout > 0 else nn.Identity()
        self.out_conv = nn.Conv3d(features[0], out_channels, kernel_size=1)
        self.engine_dtype = torch.float32
        self.kernels = "hip"

    def forward(self, x: torch.Tensor, return_features: bool = False
                ) -> Union[torch.Tensor, Tuple[torch.Tensor, List[torch.Tensor]]]:
        if self.kernels == "torch":
            check_torch_backend_input(x)
            return self.torch_forward(x, return_features)
        logits = run_engine(self, "unet", x)
        if return_features:
            prog = self.__dict__["_engine"].program
            feats = [prog.level_out(l).to_ncdhw() for l in range(len(self.features) - 1)]
            return logits, feats
        return logits

    def torch_forward(self, x: torch.Tensor, return_features: bool = False):
        """The reference forward (unet.py:165-200) over these containers in PyTorch ops."""
        x = self.init_conv(x)
        feats = [x]
        for enc in self.encoders:
            x, _ = enc(x)
            feats.append(x)
        feats = feats[:-1]
        for dec, skip in zip(self.decoders, reversed(feats)):
            x = dec(x, skip)
        x = self.out_conv(self.dropout(x))
        return (x, feats) if return_features else x

    @property
    def encoder_channels(self) -> List[int]:
        return self.features


def check_torch_backend_input(x: torch.Tensor) -> None:
    """The torch-op backend is an A/B backend on the GPU, like the HIP one: no CPU path."""
    if x.device.type != "cuda":
        raise RuntimeError("hardware.kernels: torch runs on a ROCm device; there is no CPU path")


def build_unet3d(config: Dict[str, Any]) -> UNet3D:
    """reference unet.py:208-226."""
    mc = config["model"]
    bb = mc.get("backbone", {})
    return UNet3D(in_channels=mc["in_channels"], out_channels=mc["out_channels"],
                  features=bb.get("features", [32, 64, 128, 256, 512]), norm=bb.get("norm", "instance"),
                  dropout=mc.get("head", {}).get("dropout", 0.0))
