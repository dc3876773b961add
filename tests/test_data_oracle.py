"""CPU: the data-path oracle (oracle/data_oracle.py) pinned to the reference's own transforms
(tests/golden/transforms.npz from src/data/transforms.py) and to scipy.ndimage.zoom, which the reference's
Resize calls (transforms.py:237-246)."""
import numpy as np
import pytest
from scipy.ndimage import zoom

from oracle import data_oracle as DO
from tests.helpers import golden

PRE = {"ct": {"window_center": -100, "window_width": 700}, "pet": {"normalize": True}, "mri": {"normalize": True}}


def test_normalize_reproduces_reference():
    g = golden("transforms")
    got = DO.modality_normalize(g["image_in"], ["CT", "PET", "MRI"], PRE)
    assert np.array_equal(got, g["normalized"])


@pytest.mark.parametrize("name", ["up", "down"])
def test_resize_reproduces_reference(name):
    g = golden("transforms")
    size = tuple(int(v) for v in g[f"size_{name}"])
    got = np.stack([DO.resize_linear(c, size) for c in g["normalized"]])
    assert np.array_equal(got, g[f"resized_{name}"])
    assert np.array_equal(DO.resize_nearest(g["label_in"], size), g[f"label_{name}"])


@pytest.mark.parametrize("shape,size", [((7, 9, 11), (13, 5, 11)), ((16, 16, 16), (24, 24, 24)), ((5, 4, 3), (2, 9, 3))])
def test_resize_matches_scipy(shape, size):
    rng = np.random.Generator(np.random.PCG64(3))
    v = rng.standard_normal(shape).astype(np.float32)
    zf = [o / i for o, i in zip(size, shape)]
    assert np.array_equal(DO.resize_linear(v, size), zoom(v, zf, order=1))
    lab = rng.integers(0, 7, size=shape)
    assert np.array_equal(DO.resize_nearest(lab, size), zoom(lab, zf, order=0))


def test_phantom_oracle_is_deterministic():
    a = DO.normal_stream(12345, 1000)
    assert np.array_equal(a, DO.normal_stream(12345, 1000))
    assert abs(a.mean()) < 0.15 and abs(a.std() - 1) < 0.1
    lab = DO.phantom_labels(16, np.array([[8.0, 8.0, 8.0]]), np.array([[3.0, 4.0, 5.0]]))
    assert lab[8, 8, 8] == 1 and lab[0, 0, 0] == 0
