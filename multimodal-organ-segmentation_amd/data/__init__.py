from .synthetic import SyntheticSegDataset, device_batches, phantom  # noqa: F401
from .dataloader import get_dataloader, get_dataset  # noqa: F401
from .device import (DeviceLoader, DeviceModalityNormalize, DevicePhantomDataset, DeviceResize,  # noqa: F401
                     device_phantom, phantom_params)
