"""HIP engine: runtime, layers, whole-network programs."""
from .engine import SegEngine, run_engine  # noqa: F401
