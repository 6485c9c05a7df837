"""Fixture case table shared by the oracle tests and the GPU parity tests.

Each case names the reference constructor arguments (as used by
`make_golden.py`), its deterministic input and the oracle forward to call.
"""
from __future__ import annotations

import os
from typing import Dict

import numpy as np
import torch

from detparams import det_input, det_labels, det_state_dict

HERE = os.path.dirname(os.path.abspath(__file__))

CASES = {
    "image_vit_48": dict(kind="image_vit", input_shape=(8, 3, 48, 48),
                         ctor=dict(img_size=48, patch_size=16, in_channels=3, embed_dim=384, depth=6,
                                   heads=8, mlp_dim=1536, num_classes=7, dropout=0.0)),
    "vit_base_224": dict(kind="image_vit", input_shape=(2, 3, 224, 224),
                         ctor=dict(img_size=224, patch_size=16, in_channels=3, embed_dim=768, depth=12,
                                   heads=12, mlp_dim=3072, num_classes=7, dropout=0.0)),
    "latent_vit": dict(kind="latent_vit", input_shape=(8, 18, 512),
                       ctor=dict(latent_dim=512, seq_len=18, embed_dim=512, depth=6, heads=8, mlp_dim=2048,
                                 num_classes=7, dropout=0.0)),
    "latent_vit_v2_all": dict(kind="latent_vit_v2", input_shape=(8, 18, 512),
                              ctor=dict(dropout=0.0, use_lwn=True, use_lwn_residual=True, use_spe=True,
                                        use_leam=True)),
    "latent_vit_v2_lwn": dict(kind="latent_vit_v2", input_shape=(4, 18, 512),
                              ctor=dict(dropout=0.0, depth=2, heads=4, mlp_dim=1024, use_lwn=True,
                                        use_leam=True)),
}


def load_fixture(name: str) -> Dict[str, np.ndarray]:
    with np.load(os.path.join(HERE, f"{name}.npz"), allow_pickle=False) as f:
        return {k: f[k] for k in f.files}


def fixture_state_dict(fx: Dict[str, np.ndarray]) -> Dict[str, torch.Tensor]:
    shapes = [(k, tuple(int(d) for d in s.split(",") if d != "")) for k, s in zip(fx["sd_keys"], fx["sd_shapes"])]
    return det_state_dict([(str(k), s) for k, s in shapes])


def case_inputs(name: str):
    """The case's deterministic inputs; fixtures built under the margin rule (make_golden.py
    pick_rows) name the rows they kept out of a 3x pool."""
    c = CASES[name]
    fx = load_fixture(name)
    if "input_rows" in fx:
        B = c["input_shape"][0]
        rows = torch.from_numpy(fx["input_rows"].astype(np.int64))
        x = det_input(name, (3 * B,) + tuple(c["input_shape"][1:]))[rows]
        y = det_labels(name, 3 * B)[rows]
        return x, y
    x = det_input(name, c["input_shape"])
    y = det_labels(name, c["input_shape"][0])
    return x, y


def oracle_forward(name: str, x: torch.Tensor, p: Dict[str, torch.Tensor]) -> torch.Tensor:
    import vit_oracle as O  # oracle/ is on sys.path via conftest

    c = CASES[name]
    a = c["ctor"]
    if c["kind"] == "image_vit":
        return O.image_vit_forward(x, p, a["patch_size"], a["heads"], a["depth"])
    if c["kind"] == "latent_vit":
        return O.latent_vit_forward(x, p, a["heads"], a["depth"])
    if c["kind"] == "latent_vit_v2":
        return O.latent_vit_v2_forward(x, p, a.get("heads", 8), a.get("depth", 6), a.get("use_spe", False),
                                       a.get("use_lwn", False), a.get("use_lwn_residual", False),
                                       a.get("use_leam", False))
    raise ValueError(name)


# ------------------------------------------------------------------ hybrid pieces (timm-free)
ADAPTER_KEYS = [("alpha", (1,)), ("adapter.0.weight", (64, 768)), ("adapter.0.bias", (64,)),
                ("adapter.2.weight", (768, 64)), ("adapter.2.bias", (768,))]


def adapter_inputs():
    """State dict, x [4,19,768] and dy of the `adapter` fixture (make_golden.adapter_case)."""
    sd = det_state_dict(ADAPTER_KEYS)
    sd["alpha"] = torch.tensor([0.37])
    return sd, det_input("adapter_x", (4, 19, 768)), det_input("adapter_dy", (4, 19, 768))


def check_summary(fx, key: str, t: torch.Tensor, rel: float) -> None:
    """t against a {sum, L2, samples} record: L2 and every sample within rel * L2-scale."""
    f = t.detach().reshape(-1).double().cpu()
    l2 = float(fx[key + ":l2"])
    assert abs(f.norm().item() - l2) <= rel * l2 + 1e-6, (key, f.norm().item(), l2)
    scale = l2 / max(1.0, f.numel()) ** 0.5  # rms element
    np.testing.assert_allclose(f[fx[key + ":idx"]].numpy(), fx[key + ":samples"], rtol=rel,
                               atol=rel * max(scale, 1e-6) * 4, err_msg=key)
