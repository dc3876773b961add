"""Import shim: `import mmseg_amd` loads the package directory
`multimodal-organ-segmentation_amd/` (whose name is not a Python identifier)."""
import importlib.util as _iu
import os as _os
import sys as _sys

_DIR = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "multimodal-organ-segmentation_amd")
_spec = _iu.spec_from_file_location(__name__, _os.path.join(_DIR, "__init__.py"), submodule_search_locations=[_DIR])
_mod = _iu.module_from_spec(_spec)
_sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
