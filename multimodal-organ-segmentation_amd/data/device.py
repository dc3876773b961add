"""Device-side data path: phantom generation, the reference's
ModalitySpecificNormalize (src/data/transforms.py:362-404) and Resize
(transforms.py:215-250) as HIP kernels (csrc/data.hip), and a loader that
yields batches in the reference's format (dataset.py:89-106: image, label,
patient_id, one key per modality) without touching the host.

The phantom follows data/synthetic.py's recipe (background + C-1 ellipsoid
organs; CT HU / PET SUV / MRI class intensities) with the per-sample
parameters drawn on the host from PCG64(seed + i) and the per-voxel noise from
a counter-based SplitMix64 stream on the device (oracle/data_oracle.py restates
it).  Raw volumes are then normalised by DeviceModalityNormalize with the
config's data.preprocessing, exactly as the reference's transform does on
the CPU.
"""
from __future__ import annotations

from typing import Any, Dict, Iterator, Optional, Sequence

import numpy as np
import torch

from .._lib import lib, ptr, stream_handle
from ..distributed import ddp

DEFAULT_PREPROCESSING = {"ct": {"window_center": -100, "window_width": 700}, "pet": {"normalize": True},
                         "mri": {"normalize": True}}


def _require_device(t: torch.Tensor, what: str):
    if t.device.type != "cuda":
        raise RuntimeError(f"{what}: the device data path needs ROCm tensors (got {t.device}); there is no CPU path")


class DeviceModalityNormalize:
    """transforms.py:362-404 on a [C, ...] or [B, C, ...] fp32 device tensor, in place."""

    def __init__(self, config: Dict[str, Any]):
        self.modalities = list(config["data"]["modalities"])
        self.pre = config["data"].get("preprocessing", DEFAULT_PREPROCESSING)
        self._ws = None

    def _plan(self):
        out = []
        for mod in self.modalities:
            mc = self.pre.get(mod.lower(), {})
            if mod == "CT":
                c, w = mc.get("window_center", 0), mc.get("window_width", 400)
                out.append((0, c - w / 2, c + w / 2))
            elif mod == "PET":
                out.append((1, 0.0, 0.0) if mc.get("normalize", True) else None)
            elif mod in ("MRI", "US"):
                out.append((2, 0.0, 0.0) if mc.get("normalize", True) else None)
            else:
                out.append(None)
        return out

    def __call__(self, image: torch.Tensor) -> torch.Tensor:
        _require_device(image, "DeviceModalityNormalize")
        if image.dtype != torch.float32 or not image.is_contiguous():
            raise ValueError("DeviceModalityNormalize: contiguous float32 image")
        L, s = lib(), stream_handle()
        if self._ws is None or self._ws.device != image.device:
            self._ws = torch.empty(L.mmseg_normalize_ws_bytes(), dtype=torch.uint8, device=image.device)
        C = len(self.modalities)
        if image.dim() not in (4, 5) or image.shape[-4] != C:
            raise ValueError(f"DeviceModalityNormalize: expected [{C}, D, H, W] or [B, {C}, D, H, W]")
        vols = image.reshape(-1, C, image.shape[-3] * image.shape[-2] * image.shape[-1])
        for b in range(vols.shape[0]):
            for c, step in enumerate(self._plan()):
                if step is None:
                    continue
                kind, lo, hi = step
                v = vols[b, c]
                L.mmseg_modality_normalize(ptr(v), v.numel(), kind, float(lo), float(hi), ptr(self._ws), s)
        return image


class DeviceResize:
    """transforms.py:215-250 (scipy zoom order 1 for the image, order 0 for the label) on device tensors:
    sample["image"] [C, D, H, W] fp32, sample["label"] [D, H, W] int64 / uint8 (optional)."""

    def __init__(self, size, order: int = 1):
        if order != 1:
            raise NotImplementedError("DeviceResize: order 1 (the reference default) only")
        self.size = tuple(int(v) for v in size)

    def __call__(self, sample: Dict[str, Any]) -> Dict[str, Any]:
        img = sample["image"]
        _require_device(img, "DeviceResize")
        C, D, H, W = img.shape
        d, h, w = self.size
        L, s = lib(), stream_handle()
        src = img.float().contiguous()
        out = torch.empty(C, d, h, w, dtype=torch.float32, device=img.device)
        L.mmseg_resize_linear(ptr(src), C, D, H, W, ptr(out), d, h, w, s)
        sample["image"] = out
        if "label" in sample:
            lab = sample["label"].contiguous()
            nb = lab.element_size()
            lo = torch.empty(d, h, w, dtype=lab.dtype, device=lab.device)
            L.mmseg_resize_nearest(ptr(lab), nb, 1, D, H, W, ptr(lo), d, h, w, s)
            sample["label"] = lo
        return sample


def phantom_params(seed: int, size: int, num_classes: int, modalities: Sequence[str]):
    """Host-side draws of one phantom (data/synthetic.py's distributions): geo [C-1][6] float64 (centre,
    radius), class means [M][C] float32, noise sd / |N| flag / stream key per modality."""
    rng = np.random.Generator(np.random.PCG64(seed))
    S = size
    geo = np.zeros((max(num_classes - 1, 0), 6), dtype=np.float64)
    for c in range(num_classes - 1):
        geo[c, :3] = rng.uniform(0.25 * S, 0.75 * S, 3)
        geo[c, 3:] = rng.uniform(0.08 * S, 0.22 * S, 3)
    means, sds, absn, keys = [], [], [], []
    for m, mod in enumerate(modalities):
        u = mod.upper()
        if u == "CT":
            means.append(rng.uniform(-200, 200, num_classes)); sds.append(20.0); absn.append(0)
        elif u == "PET":
            means.append(rng.uniform(0.5, 8.0, num_classes)); sds.append(0.3); absn.append(1)
        else:
            means.append(rng.uniform(0.0, 1.0, num_classes)); sds.append(0.1); absn.append(0)
        keys.append((seed * 1000003 + 7919 * (m + 1)) & ((1 << 64) - 1))
    return (geo, np.asarray(means, dtype=np.float32), np.asarray(sds, dtype=np.float32),
            np.asarray(absn, dtype=np.int32), np.asarray(keys, dtype=np.uint64))


def device_phantom(seed: int, size: int, num_classes: int, modalities: Sequence[str], device,
                   label_dtype=torch.int64):
    """One raw (un-normalised) phantom generated on the device: (image [M, S, S, S] fp32, label [S, S, S])."""
    geo, means, sds, absn, keys = phantom_params(seed, size, num_classes, modalities)
    M = len(modalities)
    image = torch.empty(M, size, size, size, dtype=torch.float32, device=device)
    label = torch.empty(size, size, size, dtype=label_dtype, device=device)
    _require_device(image, "device_phantom")
    lib().mmseg_phantom(size, geo.shape[0], geo.ctypes.data, M, means.ctypes.data, sds.ctypes.data,
                        absn.ctypes.data, keys.ctypes.data, ptr(label), label.element_size(), ptr(image),
                        stream_handle())
    return image, label


class DevicePhantomDataset:
    """Device-side counterpart of SyntheticSegDataset: sample i = phantom(seed + i) generated and normalised
    on the GPU, in the reference's batch format."""

    def __init__(self, n: int, size: int, num_classes: int, modalities: Sequence[str], device,
                 seed: int = 1234, preprocessing: Optional[Dict] = None, resize=None):
        self.n, self.size, self.C, self.mods, self.seed = n, size, num_classes, list(modalities), seed
        self.device = torch.device(device)
        self.norm = DeviceModalityNormalize({"data": {"modalities": self.mods,
                                                      "preprocessing": preprocessing or DEFAULT_PREPROCESSING}})
        self.resize = DeviceResize(resize) if resize is not None else None

    def __len__(self):
        return self.n

    def __getitem__(self, i: int) -> Dict[str, Any]:
        image, label = device_phantom(self.seed + i, self.size, self.C, self.mods, self.device)
        self.norm(image)
        sample = {"image": image, "label": label}
        if self.resize is not None:
            sample = self.resize(sample)
        sample["patient_id"] = f"synthetic_{self.seed + i}"
        for m, mod in enumerate(self.mods):
            sample[mod] = sample["image"][m]
        return sample


class DeviceLoader:
    """Batches of a DevicePhantomDataset (DistributedSampler semantics under DP: rank r takes r, r+W, ...)."""

    def __init__(self, ds: DevicePhantomDataset, batch_size: int, shuffle: bool = False, drop_last: bool = False,
                 seed: int = 0, pad: bool = True):
        self.ds, self.B, self.shuffle, self.drop_last, self.seed = ds, batch_size, shuffle, drop_last, seed
        self.epoch = 0
        # pad=True (training): equal-length shards; pad=False (validation): every sample scored once
        self.idx = (ddp.shard_indices(len(ds), ddp.rank(), ddp.world(), pad=pad) if ddp.world() > 1
                    else list(range(len(ds))))

    def __len__(self):
        n = len(self.idx)
        return n // self.B if self.drop_last else -(-n // self.B)

    def __iter__(self) -> Iterator[Dict[str, Any]]:
        order = list(self.idx)
        if self.shuffle:
            rng = np.random.Generator(np.random.PCG64(self.seed + self.epoch))
            order = [order[k] for k in rng.permutation(len(order))]
        self.epoch += 1
        for b in range(len(self)):
            items = [self.ds[i] for i in order[b * self.B:(b + 1) * self.B]]
            batch = {"image": torch.stack([it["image"] for it in items]),
                     "label": torch.stack([it["label"] for it in items]),
                     "patient_id": [it["patient_id"] for it in items]}
            for m, mod in enumerate(self.ds.mods):
                batch[mod] = batch["image"][:, m:m + 1]
            yield batch
