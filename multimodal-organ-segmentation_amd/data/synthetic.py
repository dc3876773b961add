"""Seeded synthetic CT/PET/MRI phantoms, in the reference's
batch format (dataset.py:89-106: {"image", "label", "patient_id", <modality>}).

Labels: background + C-1 random non-overlapping ellipsoid "organs".
CT : per-class HU mean in [-200, 200] + N(0, 20^2), clipped to the reference
     CT window (center -100, width 700 -> [-450, 250], default.yaml:26-27) and
     mapped to [0, 1] (transforms.py:380-387).
PET: per-class SUV in [0.5, 8] + |N(0, 0.3^2)|, divided by the max (389-394).
MRI: per-class intensity + noise, z-scored (396-401).
There is no network in this environment, so synthetic phantoms replace the
reference's NIfTI datasets for benchmarking and parity runs.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import numpy as np
import torch


def phantom(seed: int, size: int, num_classes: int, modalities: Sequence[str],
            class_seed: Optional[int] = None) -> Dict[str, np.ndarray]:
    """class_seed: None (default) draws each organ's intensities per phantom, so only shape and contrast tell the
    organs apart; an integer draws them once from that seed for every phantom ("organ-consistent" phantoms, on
    which a model learns which organ is which -- used for the held-out Dice parity set)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    crng = rng if class_seed is None else np.random.Generator(np.random.PCG64(class_seed))
    S = size
    z, y, x = np.meshgrid(*(np.arange(S, dtype=np.float32),) * 3, indexing="ij")
    label = np.zeros((S, S, S), dtype=np.int64)
    for c in range(1, num_classes):
        ctr = rng.uniform(0.25 * S, 0.75 * S, 3)
        rad = rng.uniform(0.08 * S, 0.22 * S, 3)
        inside = (((z - ctr[0]) / rad[0]) ** 2 + ((y - ctr[1]) / rad[1]) ** 2 + ((x - ctr[2]) / rad[2]) ** 2) <= 1.0
        label[inside & (label == 0)] = c
    out = {}
    for mod in modalities:
        m = mod.upper()
        if m == "CT":
            hu = crng.uniform(-200, 200, num_classes).astype(np.float32)
            img = hu[label] + rng.normal(0, 20, label.shape).astype(np.float32)
            img = (np.clip(img, -450.0, 250.0) + 450.0) / 700.0
        elif m == "PET":
            suv = crng.uniform(0.5, 8.0, num_classes).astype(np.float32)
            img = suv[label] + np.abs(rng.normal(0, 0.3, label.shape)).astype(np.float32)
            img = img / img.max()
        else:
            mu = crng.uniform(0.0, 1.0, num_classes).astype(np.float32)
            img = mu[label] + rng.normal(0, 0.1, label.shape).astype(np.float32)
            img = (img - img.mean()) / (img.std() + 1e-8)
        out[mod] = img.astype(np.float32)
    out["label"] = label
    return out


class SyntheticSegDataset(torch.utils.data.Dataset):
    """Deterministic phantom dataset: sample i is phantom(seed + i)."""

    def __init__(self, n: int, size: int, num_classes: int, modalities: Sequence[str], seed: int = 1234):
        self.n, self.size, self.C, self.mods, self.seed = n, size, num_classes, list(modalities), seed

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        p = phantom(self.seed + i, self.size, self.C, self.mods)
        item = {"image": torch.from_numpy(np.stack([p[m] for m in self.mods])),
                "label": torch.from_numpy(p["label"]), "patient_id": f"synthetic_{self.seed + i:06d}"}
        for m in self.mods:
            item[m] = torch.from_numpy(p[m][None])
        return item


def device_batches(n_batches: int, batch: int, size: int, num_classes: int, modalities: Sequence[str],
                   device, seed: int = 1234) -> List[Dict[str, torch.Tensor]]:
    """Pre-stage batches in HBM (the throughput benchmark's input path)."""
    ds = SyntheticSegDataset(n_batches * batch, size, num_classes, modalities, seed)
    out = []
    for b in range(n_batches):
        items = [ds[b * batch + j] for j in range(batch)]
        out.append({"image": torch.stack([it["image"] for it in items]).to(device),
                    "label": torch.stack([it["label"] for it in items]).to(device)})
    return out
