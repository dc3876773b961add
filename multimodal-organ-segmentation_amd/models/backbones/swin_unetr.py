"""SwinUNETR entry of the model registry (reference swin_unetr.py:20-200).

The reference wraps monai.networks.nets.SwinUNETR (swin_unetr.py:80-96) as
`self.model`; MONAI is not installed in this image, so the arithmetic is
parity-unpinned and follows MONAI 1.3's published architecture
(restated in oracle/swin_oracle.py, which the tests hold the engine to).

The modules below are parameter containers with MONAI's module tree and
state-dict names (model.swinViT.patch_embed.proj, model.swinViT.layers1.0.
blocks.0.attn.qkv, ..., model.encoder1.layer.conv1.conv, model.decoder5.
transp_conv.conv, model.out.conv.conv), so MONAI SwinUNETR checkpoints load
unchanged.  `SwinUNETR.forward` runs the whole network as one HIP program
(engine/swin.py); `WindowAttention` is also usable on its own (forward +
backward on engine/attention.py:WindowAttentionEngine).
"""
from __future__ import annotations

from typing import Any, Dict, List, Sequence, Tuple, Union

import torch
import torch.nn as nn

from ...engine import run_engine
from ...engine.attention import WindowAttentionEngine
from ...engine.runtime import Runtime


def relative_position_index(window_size: Sequence[int]) -> torch.Tensor:
    """MONAI WindowAttention.__init__ (3-D branch): index[n][m] into the
    (2w0-1)(2w1-1)(2w2-1)-row bias table for tokens n, m of one window."""
    w0, w1, w2 = window_size
    coords = torch.stack(torch.meshgrid(torch.arange(w0), torch.arange(w1), torch.arange(w2), indexing="ij"))
    flat = torch.flatten(coords, 1)
    rel = (flat[:, :, None] - flat[:, None, :]).permute(1, 2, 0).contiguous()
    rel[:, :, 0] += w0 - 1
    rel[:, :, 1] += w1 - 1
    rel[:, :, 2] += w2 - 1
    rel[:, :, 0] *= (2 * w1 - 1) * (2 * w2 - 1)
    rel[:, :, 1] *= 2 * w2 - 1
    return rel.sum(-1)


class _WindowAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mod, x, mask, qkv_w, qkv_b, proj_w, proj_b, table):
        p = {"qkv_w": qkv_w.detach().contiguous(), "proj_w": proj_w.detach().contiguous(),
             "proj_b": proj_b.detach().contiguous(), "table": table.detach().contiguous()}
        if qkv_b is not None:
            p["qkv_b"] = qkv_b.detach().contiguous()
        eng, index, csr = mod._device_state(x.device)
        y, st = eng.forward(x.float().contiguous(), None if mask is None else mask.float().contiguous(), p, index)
        ctx.mod, ctx.p, ctx.st, ctx.has_qkv_b = mod, p, st, qkv_b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        eng, _, csr = ctx.mod._device_state(dy.device)
        grads = {k: torch.empty_like(v) for k, v in ctx.p.items()}
        dx = eng.backward(dy.contiguous(), ctx.st, ctx.p, grads, csr)
        ctx.st = None
        return (None, dx, None, grads["qkv_w"], grads.get("qkv_b"), grads["proj_w"], grads["proj_b"],
                grads["table"])


class WindowAttention(nn.Module):
    """MONAI SwinUNETR WindowAttention on the engine (attention dropout / proj dropout must be 0, as in
    SwinUNETR's defaults)."""

    def __init__(self, dim: int, num_heads: int, window_size: Sequence[int], qkv_bias: bool = False,
                 attn_drop: float = 0.0, proj_drop: float = 0.0, engine_dtype: torch.dtype = torch.float32):
        super().__init__()
        if attn_drop or proj_drop:
            raise NotImplementedError("WindowAttention dropout is not on the engine (SwinUNETR uses 0)")
        self.dim, self.num_heads, self.window_size = dim, num_heads, tuple(window_size)
        self.scale = (dim // num_heads) ** -0.5
        w0, w1, w2 = self.window_size
        self.relative_position_bias_table = nn.Parameter(
            torch.zeros((2 * w0 - 1) * (2 * w1 - 1) * (2 * w2 - 1), num_heads))
        self.register_buffer("relative_position_index", relative_position_index(self.window_size))
        self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
        self.proj = nn.Linear(dim, dim)
        nn.init.trunc_normal_(self.relative_position_bias_table, std=0.02)
        self.engine_dtype = engine_dtype
        self._state = None

    def _device_state(self, device):
        if self._state is None or self._state[0].rt.device != device:
            N = self.relative_position_index.shape[0]
            idx = self.relative_position_index.reshape(-1).cpu().to(torch.int64)
            T = self.relative_position_bias_table.shape[0]
            order = torch.argsort(idx, stable=True)            # CSR of (n*N + m) per table row, ascending
            counts = torch.bincount(idx, minlength=T)
            offs = torch.zeros(T + 1, dtype=torch.int64)
            offs[1:] = torch.cumsum(counts, 0)
            csr = (offs.to(torch.int32).to(device), order.to(torch.int32).to(device), T)
            eng = WindowAttentionEngine(Runtime(device, self.engine_dtype), self.dim, self.num_heads)
            self._state = (eng, idx.to(torch.int32).to(device), csr)
            del N
        return self._state

    def forward(self, x: torch.Tensor, mask: torch.Tensor = None) -> torch.Tensor:
        n = x.shape[1]
        if n != self.relative_position_index.shape[0]:
            raise ValueError("the engine's window attention needs full windows (N = prod(window_size))")
        return _WindowAttnFn.apply(self, x, mask, self.qkv.weight, self.qkv.bias, self.proj.weight, self.proj.bias,
                                   self.relative_position_bias_table)


class _Conv(nn.Module):
    """MONAI Convolution(conv_only=True): the conv sits in child "conv"."""

    def __init__(self, conv: nn.Module):
        super().__init__()
        self.conv = conv


class UnetResBlock(nn.Module):
    """MONAI UnetResBlock(k3, stride 1, norm "instance", LeakyReLU 0.01): conv1, conv2 (no bias), IN x 2,
    and conv3 (1x1) + norm3 when the channel count changes."""

    def __init__(self, in_channels: int, out_channels: int):
        super().__init__()
        self.conv1 = _Conv(nn.Conv3d(in_channels, out_channels, 3, padding=1, bias=False))
        self.conv2 = _Conv(nn.Conv3d(out_channels, out_channels, 3, padding=1, bias=False))
        self.lrelu = nn.LeakyReLU(negative_slope=0.01, inplace=True)
        self.norm1 = nn.InstanceNorm3d(out_channels)
        self.norm2 = nn.InstanceNorm3d(out_channels)
        self.downsample = in_channels != out_channels
        if self.downsample:
            self.conv3 = _Conv(nn.Conv3d(in_channels, out_channels, 1, bias=False))
            self.norm3 = nn.InstanceNorm3d(out_channels)


class UnetrBasicBlock(nn.Module):
    def __init__(self, in_channels: int, out_channels: int):
        super().__init__()
        self.layer = UnetResBlock(in_channels, out_channels)


class UnetrUpBlock(nn.Module):
    """ConvTranspose3d(k2 s2, no bias) -> cat([up, skip]) -> UnetResBlock(2C -> C)."""

    def __init__(self, in_channels: int, out_channels: int):
        super().__init__()
        self.transp_conv = _Conv(nn.ConvTranspose3d(in_channels, out_channels, 2, stride=2, bias=False))
        self.conv_block = UnetResBlock(out_channels + out_channels, out_channels)


class UnetOutBlock(nn.Module):
    def __init__(self, in_channels: int, out_channels: int):
        super().__init__()
        self.conv = _Conv(nn.Conv3d(in_channels, out_channels, 1, bias=True))


class MLPBlock(nn.Module):
    def __init__(self, hidden_size: int, mlp_dim: int):
        super().__init__()
        self.linear1 = nn.Linear(hidden_size, mlp_dim)
        self.linear2 = nn.Linear(mlp_dim, hidden_size)
        self.fn = nn.GELU()


class SwinTransformerBlock(nn.Module):
    def __init__(self, dim: int, num_heads: int, window_size: Sequence[int], shift_size: Sequence[int],
                 mlp_ratio: float = 4.0, qkv_bias: bool = True):
        super().__init__()
        self.dim, self.num_heads = dim, num_heads
        self.window_size, self.shift_size = tuple(window_size), tuple(shift_size)
        self.norm1 = nn.LayerNorm(dim)
        self.attn = WindowAttention(dim, num_heads, self.window_size, qkv_bias=qkv_bias)
        self.drop_path = nn.Identity()
        self.norm2 = nn.LayerNorm(dim)
        self.mlp = MLPBlock(dim, int(dim * mlp_ratio))


class PatchMerging(nn.Module):
    """MONAI legacy PatchMerging ("merging"): Linear(8C -> 2C, no bias) after LayerNorm(8C)."""

    def __init__(self, dim: int):
        super().__init__()
        self.dim = dim
        self.reduction = nn.Linear(8 * dim, 2 * dim, bias=False)
        self.norm = nn.LayerNorm(8 * dim)


class BasicLayer(nn.Module):
    def __init__(self, dim: int, depth: int, num_heads: int, window_size: Sequence[int]):
        super().__init__()
        self.window_size = tuple(window_size)
        self.shift_size = tuple(i // 2 for i in window_size)
        self.no_shift = tuple(0 for _ in window_size)
        self.depth = depth
        self.blocks = nn.ModuleList([
            SwinTransformerBlock(dim, num_heads, self.window_size,
                                 self.no_shift if i % 2 == 0 else self.shift_size) for i in range(depth)])
        self.downsample = PatchMerging(dim)


class PatchEmbed(nn.Module):
    def __init__(self, patch_size: int, in_chans: int, embed_dim: int):
        super().__init__()
        self.proj = nn.Conv3d(in_chans, embed_dim, kernel_size=patch_size, stride=patch_size)


class SwinTransformer(nn.Module):
    def __init__(self, in_chans: int, embed_dim: int, window_size: Sequence[int], depths: Sequence[int],
                 num_heads: Sequence[int], drop_rate: float = 0.0):
        super().__init__()
        self.patch_embed = PatchEmbed(2, in_chans, embed_dim)
        self.pos_drop = nn.Dropout(p=drop_rate)   # applied by the engine (engine/swin.py Drop), as are the
        # blocks' proj_drop / MLP drop1 / drop2 of the same rate
        for i in range(4):
            layers = nn.ModuleList([BasicLayer(embed_dim * 2 ** i, depths[i], num_heads[i], window_size)])
            setattr(self, f"layers{i + 1}", layers)


class SwinUNETRNet(nn.Module):
    """monai.networks.nets.SwinUNETR module tree (v1.3, use_v2=False, downsample="merging")."""

    def __init__(self, in_channels: int, out_channels: int, feature_size: int, depths: Sequence[int],
                 num_heads: Sequence[int], window_size: Sequence[int] = (7, 7, 7), normalize: bool = True,
                 drop_rate: float = 0.0):
        super().__init__()
        fs = feature_size
        self.normalize = normalize
        self.swinViT = SwinTransformer(in_channels, fs, window_size, depths, num_heads, drop_rate)
        self.encoder1 = UnetrBasicBlock(in_channels, fs)
        self.encoder2 = UnetrBasicBlock(fs, fs)
        self.encoder3 = UnetrBasicBlock(2 * fs, 2 * fs)
        self.encoder4 = UnetrBasicBlock(4 * fs, 4 * fs)
        self.encoder10 = UnetrBasicBlock(16 * fs, 16 * fs)
        self.decoder5 = UnetrUpBlock(16 * fs, 8 * fs)
        self.decoder4 = UnetrUpBlock(8 * fs, 4 * fs)
        self.decoder3 = UnetrUpBlock(4 * fs, 2 * fs)
        self.decoder2 = UnetrUpBlock(2 * fs, fs)
        self.decoder1 = UnetrUpBlock(fs, fs)
        self.out = UnetOutBlock(fs, out_channels)


class SwinUNETR(nn.Module):
    """Reference SwinUNETR wrapper (swin_unetr.py:20-176): same constructor, `self.model`, forward(x,
    return_features), load_pretrained, get_encoder / get_decoder, encoder_channels.  The network runs as ONE
    HIP program (engine/swin.py).  Engine limits (raise otherwise): patch 2, 3-D, normalize=True,
    downsample="merging", use_v2=False, attention dropout / drop-path 0 (drop_rate, the reference's head.dropout,
    is supported: pos_drop, proj_drop and the MLP dropouts on the engine), feature_size / 3 heads
    -> head_dim a multiple of 8 (feature_size 24, 48, ...)."""

    def __init__(self, img_size: Tuple[int, int, int] = (96, 96, 96), in_channels: int = 1, out_channels: int = 8,
                 feature_size: int = 48, depths: Sequence[int] = (2, 2, 2, 2), num_heads: Sequence[int] = (3, 6, 12, 24),
                 norm_name: str = "instance", drop_rate: float = 0.0, attn_drop_rate: float = 0.0,
                 dropout_path_rate: float = 0.0, normalize: bool = True, use_checkpoint: bool = False,
                 spatial_dims: int = 3, downsample: str = "merging", use_v2: bool = False,
                 pretrained: str = None, **kwargs):
        super().__init__()
        if (norm_name != "instance" or attn_drop_rate or dropout_path_rate or not normalize
                or spatial_dims != 3 or downsample != "merging" or use_v2):
            raise NotImplementedError("SwinUNETR engine: norm 'instance', no attention dropout / drop-path, "
                                      "normalize=True, 3-D, downsample='merging', use_v2=False (the reference's "
                                      "build_swin_unetr defaults; drop_rate is supported)")
        if not 0.0 <= drop_rate < 1.0:
            raise ValueError(f"drop_rate must be in [0, 1), got {drop_rate}")
        self.drop_rate = float(drop_rate)
        if feature_size % 12:
            raise ValueError("feature_size should be divisible by 12 (MONAI SwinUNETR)")
        if any(s % 32 for s in img_size):
            raise ValueError("img_size dims must be divisible by 32 (MONAI SwinUNETR)")
        if len(depths) != 4 or len(num_heads) != 4:
            raise ValueError("SwinUNETR: 4 stages")
        for i, h in enumerate(num_heads):
            if ((feature_size << i) // h) % 8 or (feature_size << i) % h:
                raise NotImplementedError("SwinUNETR engine: per-stage head_dim must be a multiple of 8")
        self.img_size = tuple(img_size)
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.feature_size = feature_size
        self.num_heads = tuple(num_heads)
        self.depths = tuple(depths)
        self.window_size = (7, 7, 7)
        self.model = SwinUNETRNet(in_channels, out_channels, feature_size, depths, num_heads, self.window_size,
                                  drop_rate=self.drop_rate)
        self.engine_dtype = torch.float32
        if pretrained is not None:
            self.load_pretrained(pretrained)

    def forward(self, x: torch.Tensor, return_features: bool = False
                ) -> Union[torch.Tensor, Tuple[torch.Tensor, List[torch.Tensor]]]:
        logits = run_engine(self, "swin_unetr", x)
        if return_features:
            prog = self.__dict__["_engine"].program
            return logits, [h.to_ncdhw() for h in prog.hs]
        return logits

    def load_pretrained(self, path: str) -> None:
        state = torch.load(path, map_location="cpu", weights_only=True)
        if "model_state_dict" in state:
            state = state["model_state_dict"]
        elif "state_dict" in state:
            state = state["state_dict"]
        missing, unexpected = self.model.load_state_dict(state, strict=False)
        if missing:
            print(f"Missing keys: {len(missing)}")
        if unexpected:
            print(f"Unexpected keys: {len(unexpected)}")

    def get_encoder(self) -> nn.Module:
        return self.model.swinViT

    def get_decoder(self) -> nn.Module:
        m = self.model
        return nn.ModuleList([m.decoder5, m.decoder4, m.decoder3, m.decoder2, m.decoder1])

    @property
    def encoder_channels(self) -> List[int]:
        fs = self.feature_size
        return [fs, fs * 2, fs * 4, fs * 8, fs * 16]


def build_swin_unetr(config: Dict[str, Any]) -> SwinUNETR:
    """reference swin_unetr.py:180-200."""
    bb = config.get("model", {}).get("backbone", {})
    return SwinUNETR(img_size=tuple(bb.get("img_size", [96, 96, 96])), in_channels=config["model"]["in_channels"],
                     out_channels=config["model"]["out_channels"], feature_size=bb.get("feature_size", 48),
                     depths=tuple(bb.get("depths", [2, 2, 2, 2])), num_heads=tuple(bb.get("num_heads", [3, 6, 12, 24])),
                     drop_rate=config["model"].get("head", {}).get("dropout", 0.0),
                     use_checkpoint=config.get("training", {}).get("use_checkpoint", False))
