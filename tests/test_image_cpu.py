"""ImageViT transform oracle on the CPU (`data/image_dataset.py:139-173`): the Pillow-based
restatement reproduces the committed fixture (tests/golden/image_aug.npz, written by
make_image_golden.py), its torchvision glue matches the published formulas on known cases,
and the host packing of the GPU transform accepts the reference's image modes."""
import os

import numpy as np
import pytest
from PIL import Image

import image_oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "image_aug.npz")


def _img(a):
    return Image.fromarray(a[:, :, 0] if a.shape[2] == 1 else a, {1: "L", 3: "RGB", 4: "RGBA"}[a.shape[2]])


def test_oracle_reproduces_fixture():
    g = np.load(GOLD)
    S, n = int(g["S"]), int(g["n_src"])
    srcs = [g[f"src{i}"] for i in range(n)]
    for i, a in enumerate(srcs):
        assert np.array_equal(O.val_uint8(_img(a), S), g["val_u8"][i])
    for j, p in enumerate(g["params"]):
        assert np.array_equal(O.train_uint8(_img(srcs[j % n]), S, p), g["train_u8"][j]), j


def test_identity_record_is_resize_only():
    rng = np.random.default_rng(3)
    a = rng.integers(0, 256, (40, 50, 3), dtype=np.uint8)
    p = np.zeros(16, np.float32)
    p[O.P_BRIGHT:O.P_SAT + 1] = 1.0
    p[O.P_ORDER:O.P_ORDER + 4] = [0, 1, 2, 3]
    p[O.P_SCALE] = 1.0
    assert np.array_equal(O.train_uint8(_img(a), 32, p), O.val_uint8(_img(a), 32))


def test_affine_matrix_is_scale_translate():
    m = O.affine_matrix(224, 5, -3, 1.25)
    assert m[1] == 0 and m[3] == 0 and m[0] == m[4] == 1 / 1.25
    # inverse map: output centre -> centre - translation / scale
    assert abs((m[0] * 112 + m[2]) - (112 - 5 / 1.25)) < 1e-12 and abs((m[4] * 112 + m[5]) - (112 + 3 / 1.25)) < 1e-12


def test_normalize_matches_torchvision_formula():
    u8 = np.arange(0, 256, dtype=np.uint8).reshape(16, 16, 1).repeat(3, 2)
    x = O.normalize(u8)
    assert x.dtype == np.float32 and x.shape == (3, 16, 16)
    assert np.allclose(x[0, 0, 0], (0 - 0.485) / 0.229) and np.allclose(x[2, 15, 15], (1 - 0.406) / 0.225)


def test_host_packing_modes():
    pytest.importorskip("torch")
    from fervit.vision import _as_hwc

    g = np.zeros((5, 7), np.uint8)
    assert _as_hwc(g).shape == (5, 7, 1)
    assert _as_hwc(Image.fromarray(g, "L")).shape == (5, 7, 1)
    assert _as_hwc(np.zeros((5, 7, 4), np.uint8)).shape == (5, 7, 3)
    assert _as_hwc(Image.new("P", (7, 5))).shape == (5, 7, 3)
    with pytest.raises(TypeError):
        _as_hwc(np.zeros((5, 7, 3), np.float32))
