from .build import MODEL_REGISTRY, MultiModalSegmentationModel, build_model, get_model  # noqa: F401
from .build import load_checkpoint, save_checkpoint  # noqa: F401
