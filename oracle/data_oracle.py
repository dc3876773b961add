"""CPU oracle for the device-side data path — TEST INFRASTRUCTURE ONLY.

Only ``tests/`` use this file, as the checker.  It restates:

  * ModalitySpecificNormalize (reference src/data/transforms.py:362-404): CT window clip + scale, PET divide
    by the volume max, MRI/US z-score (numpy float32 arithmetic, std with ddof 0 and +1e-8);
  * Resize (transforms.py:215-250): scipy.ndimage.zoom(order=1) per image channel and zoom(order=0) for
    labels.  scipy 1.x's zoom with grid_mode=False maps output index o to input coordinate
    o * (in - 1) / (out - 1) (corner-aligned), interpolates linearly in float64 per axis (tensor product
    of the two neighbours, cval 0 outside — only reached with weight 0) and, for order 0, takes the nearest
    input index (half-way rounds up);
  * the device phantom generator of data/device.py: ellipsoid labels from host-drawn parameters, per-voxel
    noise from a counter-based SplitMix64 stream (key = seed, counter = voxel index per (sample,
    modality)) through Box-Muller in float64.

Pinned against tests/golden/transforms.npz (the reference's own transforms run on a raw CT/PET/MRI sample by
tests/golden/make_golden.py).  The phantom generator has no reference counterpart (the reference reads
NIfTI files); its restatement here is the definition the HIP kernel is tested against.
"""
from __future__ import annotations

from typing import Dict, Sequence

import numpy as np

MASK64 = (1 << 64) - 1


# ---------------------------------------------------------------- normalize
def modality_normalize(image: np.ndarray, modalities: Sequence[str], pre: Dict) -> np.ndarray:
    """transforms.py:374-404 on a [C, ...] float32 array (returns a copy)."""
    out = image.astype(np.float32).copy()
    for c, mod in enumerate(modalities):
        mc = pre.get(mod.lower(), {})
        if mod == "CT":
            center, width = mc.get("window_center", 0), mc.get("window_width", 400)
            lo, hi = center - width / 2, center + width / 2
            out[c] = (np.clip(out[c], lo, hi) - np.float32(lo)) / np.float32(hi - lo)
        elif mod == "PET":
            if mc.get("normalize", True):
                m = out[c].max()
                if m > 0:
                    out[c] = out[c] / m
        elif mod in ("MRI", "US"):
            if mc.get("normalize", True):
                v = out[c].astype(np.float64)
                mean, std = v.mean(), v.std() + 1e-8
                out[c] = ((out[c] - np.float32(mean)) / np.float32(std)).astype(np.float32)
    return out


# ------------------------------------------------------------------- resize
def _axis_linear(n_in: int, n_out: int):
    """Per output index: (i0, i1, w0, w1) of scipy zoom order 1, grid_mode=False."""
    z = (n_in - 1) / (n_out - 1) if n_out > 1 else 0.0
    x = np.arange(n_out, dtype=np.float64) * z
    i0 = np.floor(x).astype(np.int64)
    f = x - i0
    i1 = i0 + 1
    return i0, i1, 1.0 - f, f


def resize_linear(vol: np.ndarray, size) -> np.ndarray:
    """scipy.ndimage.zoom(vol, size / shape, order=1) restated (float64 math, float32 out)."""
    v = vol.astype(np.float64)
    for ax, n_out in enumerate(size):
        n_in = v.shape[ax]
        i0, i1, w0, w1 = _axis_linear(n_in, n_out)
        a = np.take(v, np.clip(i0, 0, n_in - 1), axis=ax)
        valid = (i1 < n_in)
        b = np.take(v, np.clip(i1, 0, n_in - 1), axis=ax)
        shp = [1] * v.ndim
        shp[ax] = n_out
        w1v = np.where(valid, w1, 0.0).reshape(shp)
        v = a * w0.reshape(shp) + b * w1v
    return v.astype(np.float32)


def resize_nearest(vol: np.ndarray, size) -> np.ndarray:
    """scipy.ndimage.zoom(vol, size / shape, order=0) restated."""
    out = vol
    for ax, n_out in enumerate(size):
        n_in = out.shape[ax]
        z = (n_in - 1) / (n_out - 1) if n_out > 1 else 0.0
        idx = np.floor(np.arange(n_out, dtype=np.float64) * z + 0.5).astype(np.int64)
        out = np.take(out, np.clip(idx, 0, n_in - 1), axis=ax)
    return out


# ------------------------------------------------------------ phantom (device)
def splitmix64(x: np.ndarray) -> np.ndarray:
    x = (x + np.uint64(0x9E3779B97F4A7C15)) & np.uint64(MASK64)
    z = x
    z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & np.uint64(MASK64)
    z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & np.uint64(MASK64)
    return z ^ (z >> np.uint64(31))


def normal_stream(key: int, n: int) -> np.ndarray:
    """Standard normals of stream `key`: element i from hash(key, i) via Box-Muller (float64)."""
    with np.errstate(over="ignore"):
        base = splitmix64(np.array([key], dtype=np.uint64))[0]
        h = splitmix64(np.arange(n, dtype=np.uint64) ^ base)
    u1 = ((h >> np.uint64(11)).astype(np.float64) + 1.0) * (1.0 / 9007199254740992.0)   # (0, 1]
    u2 = (h & np.uint64(0x1FFFFF)).astype(np.float64) * (1.0 / 2097152.0)               # [0, 1)
    return np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2)


def phantom_labels(S: int, ctr: np.ndarray, rad: np.ndarray) -> np.ndarray:
    """Class c (1..C-1) fills ellipsoid c where no earlier class did (ctr / rad [C-1][3], float64)."""
    z, y, x = np.meshgrid(*(np.arange(S, dtype=np.float64),) * 3, indexing="ij")
    label = np.zeros((S, S, S), dtype=np.int64)
    for c in range(ctr.shape[0]):
        inside = (((z - ctr[c, 0]) / rad[c, 0]) ** 2 + ((y - ctr[c, 1]) / rad[c, 1]) ** 2
                  + ((x - ctr[c, 2]) / rad[c, 2]) ** 2) <= 1.0
        label[inside & (label == 0)] = c + 1
    return label


def phantom_intensity(label: np.ndarray, cls_mean: np.ndarray, noise_std: float, key: int, absolute: bool):
    """Raw modality volume: cls_mean[label] + noise_std * N (|N| when absolute), float32."""
    nz = normal_stream(key, label.size).reshape(label.shape)
    if absolute:
        nz = np.abs(nz)
    sd = float(np.float32(noise_std))
    return (cls_mean.astype(np.float32).astype(np.float64)[label] + sd * nz).astype(np.float32)
