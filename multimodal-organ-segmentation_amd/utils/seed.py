"""set_seed — same semantics as the reference's src/utils/seed.py:12-42.
Every op on the engine path is a deterministic HIP kernel (fixed-order
reductions, no float atomics), so enabling torch's deterministic mode is safe
here (in the reference it makes the CUDA backward of MaxPool3d / NLLLoss raise,
SURVEY §0.7)."""
import os
import random

import numpy as np
import torch


def set_seed(seed: int = 42, deterministic: bool = True) -> None:
    random.seed(seed)
    np.random.seed(seed)
    os.environ["PYTHONHASHSEED"] = str(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)
    if deterministic:
        torch.backends.cudnn.deterministic = True
        torch.backends.cudnn.benchmark = False
        try:
            torch.use_deterministic_algorithms(True, warn_only=True)
        except Exception:
            pass
