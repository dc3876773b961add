"""DualEncoder on the MI355X engine — mirror of the reference's
src/models/backbones/dual_encoder.py API.

Fusion semantics follow the reference exactly (dual_encoder.py:167-199):
"concat" -> cat + 1x1 Conv3d, "add" -> sum, "attention" -> CrossModalAttention
(SE gate over modalities), and EVERY other string (including the BASELINE's
"cross_attention", "early", "late") -> mean over modalities with no
parameters.  The real Q.K^T cross-attention (CrossAttentionFusion) is not
reachable from build_model in the reference either; it lives in
models/fusion/attention_fusion.py.

`hardware.kernels: torch` runs the reference forward (dual_encoder.py:112-199,
243-254) over the same containers in PyTorch-ROCm ops (A/B backend).
"""
from __future__ import annotations

from typing import Any, Dict, List, Tuple, Union

import torch
import torch.nn as nn

from ...engine import run_engine
from .unet import ConvBlock3D, DownBlock3D, UpBlock3D, check_torch_backend_input


def fusion_kind(fusion_type: str) -> str:
    return fusion_type if fusion_type in ("concat", "add", "attention") else "mean"


class CrossModalAttention(nn.Module):
    """SE-style modality gate: AdaptiveAvgPool3d(1) over [B, M*C, ...] -> Linear(MC, MC/r) -> ReLU
    -> Linear(MC/r, M) -> Softmax -> weighted sum over M   (reference dual_encoder.py:207-254).
    Parameters live in `attention` (indices 2 and 4, as in the reference state dict)."""

    def __init__(self, channels: int, num_modalities: int, reduction: int = 4):
        super().__init__()
        self.channels = channels
        self.num_modalities = num_modalities
        mc = channels * num_modalities
        self.attention = nn.Sequential(nn.AdaptiveAvgPool3d(1), nn.Flatten(), nn.Linear(mc, mc // reduction),
                                       nn.ReLU(inplace=True), nn.Linear(mc // reduction, num_modalities),
                                       nn.Softmax(dim=1))

    def forward(self, x):
        """torch-op backend only (reference dual_encoder.py:243-254): x [B, M, C, H, W, D] -> [B, C, H, W, D]."""
        B, M, C = x.shape[:3]
        w = self.attention(x.reshape(B, M * C, *x.shape[3:]))
        return (x * w.view(B, M, 1, 1, 1, 1)).sum(dim=1)


class DualEncoder(nn.Module):
    """Per-modality UNet encoders + per-level fusion + shared UNet decoder (reference dual_encoder.py:15-204)."""

    def __init__(self, in_channels_per_modality: int = 1, num_modalities: int = 2, out_channels: int = 8,
                 features: List[int] = (32, 64, 128, 256, 512), norm: str = "instance", fusion_type: str = "concat",
                 dropout: float = 0.0, shared_decoder: bool = True, **kwargs):
        super().__init__()
        if in_channels_per_modality != 1:
            raise NotImplementedError("engine DualEncoder: one channel per modality (reference builder default)")
        features = [int(f) for f in features]
        self.in_channels_per_modality = in_channels_per_modality
        self.num_modalities = num_modalities
        self.out_channels = out_channels
        self.features = features
        self.fusion_type = fusion_type
        self.fusion_kind = fusion_kind(fusion_type)
        self.shared_decoder = shared_decoder
        self.dropout_p = float(dropout)
        # RNG order: every encoder, then fusion layers, then decoder, then head (dual_encoder.py:58-84)
        self.encoders = nn.ModuleList([self._encoder(features, norm) for _ in range(num_modalities)])
        if fusion_type == "attention":
            self.fusion_layers = nn.ModuleList([CrossModalAttention(f, num_modalities) for f in features])
        elif fusion_type == "concat":
            self.fusion_proj = nn.ModuleList([nn.Conv3d(f * num_modalities, f, kernel_size=1) for f in features])
        self.decoder = nn.ModuleList(
            [UpBlock3D(features[i], features[i - 1], norm=norm) for i in range(len(features) - 1, 0, -1)])
        self.dropout = nn.Dropout3d(dropout) if dropout > 0 else nn.Identity()
        self.out_conv = nn.Conv3d(features[0], out_channels, kernel_size=1)
        self.engine_dtype = torch.float32
        self.kernels = "hip"

    @staticmethod
    def _encoder(features: List[int], norm: str) -> nn.ModuleDict:
        enc = nn.ModuleDict()
        enc["init_conv"] = ConvBlock3D(1, features[0], norm=norm)
        enc["blocks"] = nn.ModuleList([DownBlock3D(a, b, norm=norm) for a, b in zip(features[:-1], features[1:])])
        return enc

    def forward(self, x: torch.Tensor, return_features: bool = False
                ) -> Union[torch.Tensor, Tuple[torch.Tensor, Dict[str, List]]]:
        if self.kernels == "torch":
            check_torch_backend_input(x)
            return self.torch_forward(x, return_features)
        logits = run_engine(self, "dual_encoder", x)
        if return_features:
            prog = self.__dict__["_engine"].program
            prog.materialize_features()
            enc = [[prog.y[m][l].to_ncdhw() for l in range(len(self.features))] for m in range(self.num_modalities)]
            fused = [prog.fused_out(l).to_ncdhw() for l in range(len(self.features))]
            return logits, {"encoder_features": enc, "fused_features": fused}
        return logits

    def torch_forward(self, x: torch.Tensor, return_features: bool = False):
        """The reference forward (dual_encoder.py:112-199) over these containers in PyTorch ops."""
        allf = []
        for i, enc in enumerate(self.encoders):
            f = enc["init_conv"](x[:, i:i + 1])
            mf = [f]
            for blk in enc["blocks"]:
                f, _ = blk(f)
                mf.append(f)
            allf.append(mf)
        fused = []
        for l in range(len(allf[0])):
            lf = [f[l] for f in allf]
            if self.fusion_type == "concat":
                fused.append(self.fusion_proj[l](torch.cat(lf, dim=1)))
            elif self.fusion_type == "add":
                fused.append(sum(lf))
            elif self.fusion_type == "attention":
                fused.append(self.fusion_layers[l](torch.stack(lf, dim=1)))
            else:
                fused.append(torch.stack(lf).mean(dim=0))
        h = fused[-1]
        for dec, skip in zip(self.decoder, reversed(fused[:-1])):
            h = dec(h, skip)
        h = self.out_conv(self.dropout(h))
        if return_features:
            return h, {"encoder_features": allf, "fused_features": fused}
        return h

    @property
    def encoder_channels(self) -> List[int]:
        return self.features


def build_dual_encoder(config: Dict[str, Any]) -> DualEncoder:
    """reference dual_encoder.py:257-280."""
    mc = config["model"]
    bb = mc.get("backbone", {})
    return DualEncoder(in_channels_per_modality=1, num_modalities=len(config["data"]["modalities"]),
                       out_channels=mc["out_channels"], features=bb.get("features", [32, 64, 128, 256, 512]),
                       norm=bb.get("norm", "instance"), fusion_type=mc.get("fusion", {}).get("type", "concat"),
                       dropout=mc.get("head", {}).get("dropout", 0.0))
