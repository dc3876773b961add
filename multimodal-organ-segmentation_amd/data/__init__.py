from .synthetic import SyntheticSegDataset, device_batches, phantom  # noqa: F401
