"""Deterministic weights / inputs for parity fixtures (test infrastructure).

Every tensor is drawn from numpy's PCG64 seeded by crc32(state_dict key) ^ seed,
so the fixture generator (run once, in the build container, against the
reference) and the GPU-box tests (no reference present) rebuild bit-identical
weights from the key names alone.
"""
from __future__ import annotations

import zlib
from typing import Dict, Iterable, Tuple

import numpy as np
import torch

LAYER_GROUPS = [0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1, 2, 2, 2, 2, 2, 2]


def _rng(key: str, seed: int) -> np.random.Generator:
    return np.random.default_rng((zlib.crc32(key.encode()) ^ (seed * 0x9E3779B1)) & 0xFFFFFFFF)


def det_tensor(key: str, shape: Tuple[int, ...], seed: int = 0) -> torch.Tensor:
    """Value distribution picked from the key's role so activations stay O(1)."""
    g = _rng(key, seed)
    n = g.standard_normal(shape).astype(np.float32)
    leaf = key.rsplit(".", 1)[-1]
    if key.endswith("spe.groups") or key.endswith("groups"):
        return torch.tensor(LAYER_GROUPS[: shape[0]], dtype=torch.long)
    if leaf in ("layer_weights",):                       # LEAM raw weights
        return torch.from_numpy(0.5 + 0.6 * n)
    if leaf == "gate":                                    # LWN residual gate
        return torch.from_numpy(-0.5 + 0.8 * n)
    if leaf == "alpha":                                   # adapter alpha
        return torch.from_numpy(0.1 + 0.05 * n)
    if "norm" in key and leaf == "weight" and len(shape) == 1:
        return torch.from_numpy(1.0 + 0.1 * n)
    if ("norm" in key or key.startswith("head.0") or "mlp_head.0" in key) and leaf == "bias":
        return torch.from_numpy(0.1 * n)
    if key.endswith("mlp_head.0.weight") or key.endswith("head.0.weight"):
        return torch.from_numpy(1.0 + 0.1 * n)
    if leaf in ("cls_token", "pos_embed", "pos_emb"):
        return torch.from_numpy(0.5 * n)
    if "embed.weight" in key:                             # SPE embeddings
        return torch.from_numpy(0.5 * n)
    if leaf == "bias" or leaf.endswith("_bias"):
        return torch.from_numpy(0.02 * n)
    if len(shape) >= 2:
        fan_in = int(np.prod(shape[1:]))
        return torch.from_numpy(n / np.sqrt(fan_in))
    return torch.from_numpy(0.02 * n)


def det_state_dict(shapes: Iterable[Tuple[str, Tuple[int, ...]]], seed: int = 0) -> Dict[str, torch.Tensor]:
    out = {}
    for k, s in shapes:
        t = det_tensor(k, tuple(s), seed)
        out[k] = t if t.dtype == torch.long else t.float()
    return out


def det_input(name: str, shape: Tuple[int, ...], seed: int = 0) -> torch.Tensor:
    return torch.from_numpy(_rng("input:" + name, seed).standard_normal(shape).astype(np.float32))


def det_labels(name: str, n: int, classes: int = 7, seed: int = 0) -> torch.Tensor:
    return torch.from_numpy(_rng("labels:" + name, seed).integers(0, classes, n).astype(np.int64))


def det_directions(C: int, L: int, D: int, seed: int = 0) -> torch.Tensor:
    """Synthetic stand-in for `*_directions.pt` (`latent_analysis/compute_expression_direction.py:119-142`)."""
    return torch.from_numpy(_rng("directions", seed).standard_normal((C, L, D)).astype(np.float32))
