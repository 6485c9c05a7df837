"""LatentDecomposer (reference `models_fer_vit/latent_decomposer.py:30-174`): projection of
w+ onto fixed (buffer) expression directions. coeff = W D^T, w_expr = coeff D (or the
max-|coeff| direction only), w_id = W - w_expr. Runs fer_decompose (scores kernel + output
kernel); the directions are data, so no gradient flows through it."""
from typing import Dict, Literal

import torch
import torch.nn as nn

from fervit import ops
from fervit._lib import check, lib

EMOTION_NAMES = {0: "angry", 1: "disgust", 2: "fear", 3: "happy", 4: "neutral", 5: "sad", 6: "surprise"}
_OMODE = {"expr_only": 0, "id_only": 1, "enhanced": 2, "concat": 3}
_DMODE = {"all_classes": 0, "max_class": 1}


class LatentDecomposer(nn.Module):
    def __init__(self, directions: Dict[int, torch.Tensor], seq_len: int = 18, latent_dim: int = 512):
        super().__init__()
        self.seq_len = seq_len
        self.latent_dim = latent_dim
        self.num_classes = len(directions)
        dirs = torch.stack([directions[i] for i in range(self.num_classes)], dim=0)
        f = dirs.view(self.num_classes, -1)
        f = f / (f.norm(dim=1, keepdim=True) + 1e-12)
        self.register_buffer("directions", f.view(self.num_classes, seq_len, latent_dim))

    @classmethod
    def from_file(cls, path: str) -> "LatentDecomposer":
        """`latent_decomposer.py:67-80`, with a non-executing loader (weights_only)."""
        data = torch.load(path, map_location="cpu", weights_only=True)
        directions = data["directions"]
        seq_len = data.get("seq_len", 18)
        latent_dim = data.get("latent_dim", 512)
        print(f"Loaded '{data.get('method', 'unknown')}' expression directions: {path}")
        print(f"  Classes  : {list(directions.keys())}")
        print(f"  Direction shape: ({seq_len}, {latent_dim}) x {len(directions)} classes")
        return cls(directions, seq_len, latent_dim)

    def _run(self, w_plus, output_mode, alpha, decompose_mode, want_y=True):
        w = w_plus.contiguous().float()
        if not w.is_cuda:
            raise RuntimeError("fervit: LatentDecomposer needs a ROCm device (no CPU path)")
        B = w.shape[0]
        LD = self.seq_len * self.latent_dim
        L = self.seq_len * (2 if output_mode == "concat" else 1)
        y = torch.empty(B, L, self.latent_dim, dtype=torch.float32, device=w.device) if want_y else None
        scores = torch.empty(B, self.num_classes, dtype=torch.float32, device=w.device)
        check(lib().fer_decompose(w.data_ptr(), self.directions.data_ptr(), B, self.num_classes, LD,
                                  _OMODE[output_mode], float(alpha), _DMODE[decompose_mode], ops.ptr(y),
                                  scores.data_ptr(), ops.stream()), "decompose")
        return y, scores

    def decompose(self, w_plus: torch.Tensor, mode: Literal["all_classes", "max_class"] = "all_classes"):
        e, _ = self._run(w_plus, "expr_only", 1.0, mode)
        return e, w_plus.float() - e

    def get_expression_scores(self, w_plus: torch.Tensor) -> torch.Tensor:
        return self._run(w_plus, "expr_only", 1.0, "all_classes", want_y=False)[1]

    def enhance_expression(self, w_plus, alpha: float = 2.0, mode="all_classes"):
        return self._run(w_plus, "enhanced", alpha, mode)[0]

    def forward(self, w_plus, output_mode="expr_only", enhance_alpha: float = 2.0, decompose_mode="all_classes"):
        if output_mode not in _OMODE:
            raise ValueError(f"Unknown output_mode: {output_mode!r}")
        if decompose_mode not in _DMODE:
            raise ValueError(f"Unknown mode: {decompose_mode!r}")
        return self._run(w_plus, output_mode, enhance_alpha, decompose_mode)[0]
