"""get_dataloader(config, split) — reference src/data/dataloader.py:14-60.

The reference reads a CSV of NIfTI files (nibabel, absent here); the engine's
loader serves the seeded synthetic phantoms of data/synthetic.py in the same
batch format.  Under data parallelism each rank takes samples r, r+W, ...
(DistributedSampler semantics).  With data.synthetic.device: true
the phantoms are generated and normalised on the GPU instead (data/device.py)."""
from typing import Any, Dict

import torch
from torch.utils.data import DataLoader, Subset

from ..distributed import ddp
from .synthetic import SyntheticSegDataset


def get_dataset(config: Dict[str, Any], split: str = "train"):
    syn = config["data"].get("synthetic")
    if syn is None:
        raise NotImplementedError("NIfTI/CSV datasets are outside the engine's scope (nibabel is not available); "
                                  "set data.synthetic: {n_train, n_val, size, seed}")
    n = syn["n_train"] if split == "train" else syn.get("n_val", 2)
    seed = syn.get("seed", 1234) + (0 if split == "train" else 100000)
    return SyntheticSegDataset(n, syn.get("size", 96), config["model"]["out_channels"], config["data"]["modalities"],
                               seed=seed)


def get_dataloader(config: Dict[str, Any], split: str = "train", shuffle=None, drop_last=None):
    syn = config["data"].get("synthetic") or {}
    if syn.get("device", False):
        # data.synthetic.device: true -> phantoms generated and normalised on the GPU (data/device.py)
        from .device import DeviceLoader, DevicePhantomDataset
        n = syn["n_train"] if split == "train" else syn.get("n_val", 2)
        seed = syn.get("seed", 1234) + (0 if split == "train" else 100000)
        ds = DevicePhantomDataset(n, syn.get("size", 96), config["model"]["out_channels"],
                                  config["data"]["modalities"], torch.device("cuda", torch.cuda.current_device()),
                                  seed=seed, preprocessing=config["data"].get("preprocessing"))
        return DeviceLoader(ds, config["training"]["batch_size"],
                            shuffle=split == "train" if shuffle is None else shuffle,
                            drop_last=split == "train" if drop_last is None else drop_last, seed=seed,
                            pad=split == "train")
    ds = get_dataset(config, split)
    w, r = ddp.world(), ddp.rank()
    if w > 1:   # training shards are padded to equal length, validation shards are not (each sample once)
        ds = Subset(ds, ddp.shard_indices(len(ds), r, w, pad=split == "train"))
    if shuffle is None:
        shuffle = split == "train"
    if drop_last is None:
        drop_last = split == "train"
    hw = config.get("hardware", {})
    nw = hw.get("num_workers", 0)
    return DataLoader(ds, batch_size=config["training"]["batch_size"], shuffle=shuffle, num_workers=nw,
                      pin_memory=hw.get("pin_memory", True) and torch.cuda.is_available(), drop_last=drop_last,
                      persistent_workers=nw > 0)
