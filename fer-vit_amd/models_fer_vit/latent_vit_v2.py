"""LatentViTv2 (reference `models_fer_vit/latent_vit_v2.py:7-101`): LatentViT with an
optional w+ prologue applied in the order SPE -> LWN -> LEAM (`:82-84`), fused into one
HIP kernel pair (fer_wplus_fwd/bwd)."""
import torch
import torch.nn as nn

from fervit.module import FerModule
from modules import LEAM, LayerWiseNorm, SemanticPE
from modules._wplus import WplusSpec

from .latent_vit import LatentViT


class LatentViTv2(FerModule):
    def __init__(self, latent_dim: int = 512, seq_len: int = 18, embed_dim: int = 512, depth: int = 6,
                 heads: int = 8, mlp_dim: int = 2048, num_classes: int = 7, dropout: float = 0.1,
                 use_lwn: bool = False, use_lwn_residual: bool = False, use_spe: bool = False,
                 use_leam: bool = False):
        super().__init__()
        self.lwn = LayerWiseNorm(seq_len, latent_dim, use_residual=use_lwn_residual) if use_lwn else nn.Identity()
        self.spe = SemanticPE(latent_dim, seq_len) if use_spe else nn.Identity()
        self.leam = LEAM(seq_len) if use_leam else nn.Identity()
        self.backbone = LatentViT(latent_dim=latent_dim, seq_len=seq_len, embed_dim=embed_dim, depth=depth,
                                  heads=heads, mlp_dim=mlp_dim, num_classes=num_classes, dropout=dropout)
        self.use_lwn = use_lwn
        self.use_lwn_residual = use_lwn_residual
        self.use_spe = use_spe
        self.use_leam = use_leam

    def _spec(self):
        return WplusSpec(spe=self.spe if self.use_spe else None, lwn=self.lwn if self.use_lwn else None,
                         leam=self.leam if self.use_leam else None)

    def forward(self, w_plus: torch.Tensor) -> torch.Tensor:
        flat = self.fer_flat()
        x = w_plus
        if self.use_spe or self.use_lwn or self.use_leam:
            spec = self._spec()
            x = spec.run(w_plus, flat, self.need_grad(w_plus, spec.params()))
        return self.backbone(x)

    def get_leam_weights(self):
        """`latent_vit_v2.py:87-91`."""
        return self.leam.get_weights() if self.use_leam else None

    def get_config(self) -> dict:
        """`latent_vit_v2.py:93-101`."""
        return {"model": "LatentViTv2", "use_lwn": self.use_lwn, "use_lwn_residual": self.use_lwn_residual,
                "use_spe": self.use_spe, "use_leam": self.use_leam}
