"""YAML config loading (reference src/utils/io.py:15-33), safe loader only."""
from typing import Any, Dict

import yaml


def load_config(path: str) -> Dict[str, Any]:
    with open(path) as f:
        return yaml.safe_load(f)
