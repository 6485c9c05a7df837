"""GPU parity of the ImageViT transforms (`fer_image_augment`, csrc/image.hip) against Pillow
(oracle/image_oracle.py, the reference's `data/image_dataset.py:139-173` pipeline): the
committed fixture, live Pillow runs at the reference's 224x224 size, the hue conversion over
every 24-bit colour, and the device parameter draw. Bar: bit-exact (uint8 stages equal, so the
normalised fp32 outputs are equal)."""
import numpy as np
import pytest
import torch
from PIL import Image

import image_oracle as O

pytestmark = pytest.mark.gpu
GOLD = __file__.rsplit("/", 1)[0] + "/golden/image_aug.npz"


def _img(a):
    return Image.fromarray(a[:, :, 0] if a.shape[2] == 1 else a, {1: "L", 3: "RGB", 4: "RGBA"}[a.shape[2]])


def _norm(u8s):
    return torch.from_numpy(np.stack([O.normalize(u) for u in u8s]))


def _mismatch(out, ref):
    return int((out.cpu() != ref).sum())


def test_fixture_val_and_train_bit_exact():
    from fervit.vision import GPUImageTransform

    g = np.load(GOLD)
    S, n = int(g["S"]), int(g["n_src"])
    srcs = [g[f"src{i}"] for i in range(n)]
    val = GPUImageTransform(S, train=False)(srcs)
    assert _mismatch(val, _norm(g["val_u8"])) == 0
    P = g["params"]
    imgs = [srcs[j % n] for j in range(len(P))]
    tr = GPUImageTransform(S, train=True)(imgs, params=torch.from_numpy(P).cuda())
    assert _mismatch(tr, _norm(g["train_u8"])) == 0


@pytest.mark.parametrize("seed", [0, 1])
def test_live_pillow_224(seed):
    from fervit.vision import GPUImageTransform

    rng = np.random.default_rng(seed)
    shapes = [(48, 48, 1), (48, 48, 3), (260, 300, 3), (224, 224, 3), (120, 97, 3), (500, 380, 3)]
    srcs = [rng.integers(0, 256, s, dtype=np.uint8) for s in shapes]
    P = O.random_params(len(srcs), 224, rng)
    out = GPUImageTransform(224, train=True)(srcs, params=torch.from_numpy(P).cuda())
    ref = _norm([O.train_uint8(_img(a), 224, p) for a, p in zip(srcs, P)])
    assert _mismatch(out, ref) == 0
    val = GPUImageTransform(224, train=False)(srcs)
    assert _mismatch(val, _norm([O.val_uint8(_img(a), 224) for a in srcs])) == 0


def test_hue_every_colour():
    """All 2^24 RGB values through the hue path only (identity geometry, unit factors)."""
    from fervit.vision import GPUImageTransform

    a = np.arange(1 << 24, dtype=np.int64)
    px = np.stack([(a >> 16) & 255, (a >> 8) & 255, a & 255], -1).astype(np.uint8).reshape(16, 1024, 1024, 3)
    for hf in (-0.1, 0.0371):
        P = np.zeros((16, 16), np.float32)
        P[:, O.P_BRIGHT:O.P_SAT + 1] = 1.0
        P[:, O.P_HUE] = hf
        P[:, O.P_ORDER:O.P_ORDER + 4] = [3, 0, 1, 2]
        P[:, O.P_SCALE] = 1.0
        P[:, O.P_HUE_ON] = 1.0
        out = GPUImageTransform(1024, train=True)(list(px), params=torch.from_numpy(P).cuda())
        bad = 0
        for i in range(16):
            ref = torch.from_numpy(O.normalize(np.asarray(O.adjust_hue(Image.fromarray(px[i]), float(np.float32(hf))))))
            bad += _mismatch(out[i], ref)
        assert bad == 0, (hf, bad)


def test_device_draw_ranges_and_replay():
    from fervit import runtime
    from fervit.vision import GPUImageTransform

    rng = np.random.default_rng(7)
    srcs = [rng.integers(0, 256, (64, 80, 3), dtype=np.uint8) for _ in range(512)]
    t = GPUImageTransform(32, train=True)
    runtime.manual_seed(11)
    out = t(srcs)
    P = t.last_params.cpu().numpy()
    assert 0.4 < P[:, O.P_FLIP].mean() < 0.6 and set(np.unique(P[:, O.P_FLIP])) <= {0.0, 1.0}
    assert np.all(np.abs(P[:, O.P_ANGLE]) <= 15) and P[:, O.P_ANGLE].std() > 7
    for k, r in ((O.P_BRIGHT, 0.2), (O.P_CONTRAST, 0.2), (O.P_SAT, 0.2), (O.P_HUE, 0.1)):
        c = 0.0 if k == O.P_HUE else 1.0
        assert np.all(np.abs(P[:, k] - c) <= r + 1e-6)
    assert all(sorted(row) == [0, 1, 2, 3] for row in P[:, O.P_ORDER:O.P_ORDER + 4].astype(int).tolist())
    assert np.all(P[:, [O.P_TX, O.P_TY]] == np.round(P[:, [O.P_TX, O.P_TY]]))
    assert np.all(np.abs(P[:, [O.P_TX, O.P_TY]]) <= 4) and np.all((P[:, O.P_SCALE] >= 0.9) & (P[:, O.P_SCALE] <= 1.1))
    assert np.all(P[:, O.P_HUE_ON] == 1)
    # the drawn records reproduce the output through Pillow
    ref = _norm([O.train_uint8(_img(srcs[i]), 32, P[i]) for i in range(0, 512, 37)])
    assert _mismatch(out[0:512:37], ref) == 0
    # same seed -> same batch; next call draws new records
    runtime.manual_seed(11)
    assert torch.equal(t(srcs), out)
    assert not torch.equal(t(srcs), out)


def test_feeds_image_vit_forward():
    """The transform's output is the ImageViT input (`image_vit.py` patch embedding)."""
    from fervit.vision import get_train_transforms, get_val_transforms
    from models_fer_vit.image_vit import ImageViT

    rng = np.random.default_rng(3)
    srcs = [rng.integers(0, 256, (48, 48), dtype=np.uint8) for _ in range(4)]
    x = get_train_transforms(224)(srcs)
    assert x.shape == (4, 3, 224, 224) and x.dtype == torch.float32 and torch.isfinite(x).all()
    xv = get_val_transforms(224)(srcs)
    assert xv.abs().max() < 3.0
    m = ImageViT(img_size=224, embed_dim=192, depth=2, heads=3, mlp_dim=768).cuda().eval()
    with torch.no_grad():
        lg = m(xv)
    assert lg.shape == (4, 7) and torch.isfinite(lg).all()
