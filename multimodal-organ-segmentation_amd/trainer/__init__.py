from .losses import DiceLoss, DiceCELoss, TverskyLoss, CrossEntropyLoss, get_loss  # noqa: F401
from .metrics import DiceMetric, get_metrics  # noqa: F401
from .optim import FlatAdamW  # noqa: F401
from .trainer import Trainer  # noqa: F401
