from .seed import set_seed  # noqa: F401
from .io import load_config  # noqa: F401
from .logger import setup_logger  # noqa: F401
