"""bench.py against another in-tree build of the same ABI (A/B of two library builds in one GPU call):
    python tools/benchlib.py LIB.so [bench.py arguments ...]"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mmseg_amd import _lib  # noqa: E402

_lib.set_library_path(os.path.abspath(sys.argv[1]))
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")
