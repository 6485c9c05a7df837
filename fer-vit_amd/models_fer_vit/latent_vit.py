"""LatentViT (reference `models_fer_vit/latent_vit.py:5-48`): ViT over StyleGAN w+ tokens.

input_proj Linear(latent_dim, E) + CLS + pos_emb (randn, no custom init), post-norm
ReLU encoder (nn.TransformerEncoderLayer default activation), mlp_head = LN + Linear.
"""
import torch
import torch.nn as nn

from fervit.blocks import Encoder, EncoderLayer
from fervit.layers import HeadFn, LatentTokensFn, LayerCfg
from fervit.module import FerModule


class LatentViT(FerModule):
    def __init__(self, latent_dim: int = 512, seq_len: int = 18, embed_dim: int = 512, depth: int = 6,
                 heads: int = 8, mlp_dim: int = 2048, num_classes: int = 7, dropout: float = 0.1) -> None:
        super().__init__()
        self.seq_len = seq_len
        self.input_proj = nn.Linear(latent_dim, embed_dim)
        self.cls_token = nn.Parameter(torch.randn(1, 1, embed_dim))
        self.pos_emb = nn.Parameter(torch.randn(1, seq_len + 1, embed_dim))
        layer = EncoderLayer(embed_dim, heads, mlp_dim, dropout, activation="relu")
        self.transformer = Encoder(layer, num_layers=depth)
        self.mlp_head = nn.Sequential(nn.LayerNorm(embed_dim), nn.Linear(embed_dim, num_classes))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """x: (B, L, latent_dim) fp32 -> logits (B, num_classes)."""
        B, L, _ = x.shape
        flat = self.fer_flat()
        save = self.need_grad(x, list(self.parameters()))
        N = L + 1
        cfg = LayerCfg(B=B, N=N, H=1, save=save)
        t = LatentTokensFn.apply(x, cfg, flat, self.compute_dtype(), self.input_proj.weight, self.input_proj.bias,
                                 self.cls_token, self.pos_emb)
        t = self.transformer.run_rows(t, B, N, save)
        ln, lin = self.mlp_head[0], self.mlp_head[1]
        hcfg = LayerCfg(B=B, N=N, H=1, eps=ln.eps, save=save)
        return HeadFn.apply(t, hcfg, flat, ln.weight, ln.bias, lin.weight, lin.bias)
