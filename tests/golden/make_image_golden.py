"""Generate tests/golden/image_aug.npz: inputs and expected outputs of the ImageViT transforms
(`data/image_dataset.py:139-173`) computed by Pillow through oracle/image_oracle.py.

    python tests/golden/make_image_golden.py

Sources cover the reference's inputs: a 48x48 greyscale FER2013-style face (converted to RGB),
RGB images smaller and larger than the target (upscale / antialiased shrink), an RGBA image.
Parameter records include random torchvision-range draws and edge records (no rotation,
extreme jitter factors, hue wrapping both ways, maximum translation). Expected outputs are the
uint8 images right before ToTensor; the tests normalise both sides identically.
"""
from __future__ import annotations

import os
import sys

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import image_oracle as O  # noqa: E402

S = 64


def sources(rng):
    yy, xx = np.mgrid[0:48, 0:48]
    face = ((xx * 5 + yy * 3) % 256).astype(np.uint8)  # structured grey
    face[10:20, 12:36] = rng.integers(0, 256, (10, 24), dtype=np.uint8)
    return [
        ("grey48", face[:, :, None]),
        ("rgb37x53", rng.integers(0, 256, (37, 53, 3), dtype=np.uint8)),
        ("rgb150x170", rng.integers(0, 256, (150, 170, 3), dtype=np.uint8)),
        ("rgb64", rng.integers(0, 256, (64, 64, 3), dtype=np.uint8)),
        ("rgba70x40", rng.integers(0, 256, (70, 40, 4), dtype=np.uint8)),
        ("rgb300x90", rng.integers(0, 256, (300, 90, 3), dtype=np.uint8)),
    ]


def edge_params():
    P = np.zeros((6, 16), dtype=np.float32)
    P[:, O.P_SCALE] = 1.0
    P[:, O.P_BRIGHT:O.P_SAT + 1] = 1.0
    P[:, O.P_ORDER:O.P_ORDER + 4] = [0, 1, 2, 3]
    P[1:, O.P_HUE_ON] = 1.0  # record 0: the identity (hue disabled) -> Resize only
    P[1, [O.P_FLIP, O.P_ANGLE]] = [1, 15.0]  # flip + max rotation, no jitter
    P[2, O.P_BRIGHT:O.P_HUE + 1] = [0.8, 1.2, 0.8, -0.1]  # jitter extremes, hue wraps down
    P[2, O.P_ORDER:O.P_ORDER + 4] = [3, 2, 1, 0]
    P[3, O.P_BRIGHT:O.P_HUE + 1] = [1.2, 0.8, 1.2, 0.1]
    P[3, O.P_ORDER:O.P_ORDER + 4] = [1, 3, 0, 2]
    P[4, [O.P_TX, O.P_TY, O.P_SCALE]] = [6, -6, 0.9]  # max translation, zoom out
    P[5, [O.P_ANGLE, O.P_TX, O.P_TY, O.P_SCALE]] = [-15.0, -6, 6, 1.1]
    return P


def main():
    rng = np.random.default_rng(20261016)
    srcs = sources(rng)
    P = np.concatenate([edge_params(), O.random_params(len(srcs) * 2, S, rng)])
    out = {"S": np.int32(S), "params": P}
    val, train = [], []
    for i, (name, a) in enumerate(srcs):
        out[f"src{i}"] = a
        im = Image.fromarray(a[:, :, 0] if a.shape[2] == 1 else a, {1: "L", 3: "RGB", 4: "RGBA"}[a.shape[2]])
        val.append(O.val_uint8(im, S))
    for j in range(len(P)):
        a = srcs[j % len(srcs)][1]
        im = Image.fromarray(a[:, :, 0] if a.shape[2] == 1 else a, {1: "L", 3: "RGB", 4: "RGBA"}[a.shape[2]])
        train.append(O.train_uint8(im, S, P[j]))
    out["val_u8"] = np.stack(val)
    out["train_u8"] = np.stack(train)
    out["n_src"] = np.int32(len(srcs))
    np.savez_compressed(os.path.join(HERE, "image_aug.npz"), **out)
    print("wrote image_aug.npz:", len(srcs), "sources,", len(P), "train records")


if __name__ == "__main__":
    main()
