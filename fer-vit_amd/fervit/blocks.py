"""Parameter containers + forwards for the transformer blocks.

The containers reproduce the reference modules' parameter names, shapes and
initialisation so state_dicts interoperate with the reference's checkpoints and
eval scripts (`eval/evaluate_model.py:30-132`):
  * EncoderLayer  == nn.TransformerEncoderLayer(batch_first=True, norm_first=False)
                     keys self_attn.{in_proj_weight,in_proj_bias,out_proj.*}, linear1/2, norm1/2
  * Encoder       == nn.TransformerEncoder(layer, num_layers): `layers.{i}`, layers are
                     deep copies of one prototype (so they start identical, as in torch)
  * Block         == timm 1.0.17 vision_transformer.Block: norm1, attn.{qkv,proj}, norm2, mlp.{fc1,fc2}
  * AdapterModule == `hybrid_latent_vit.py:249-265`
Their forwards run the fused HIP layer functions in fervit.layers.
"""
from __future__ import annotations

import copy
import math

import torch
import torch.nn as nn

from .layers import AdapterFn, LayerCfg, PostNormLayerFn, PreNormBlockFn
from .module import FerModule


def _as_rows(x: torch.Tensor):
    if x.dim() == 3:
        B, N, D = x.shape
        return x.reshape(B * N, D), B, N
    raise ValueError("expected [B, N, D] tokens")


class MultiheadAttentionParams(nn.Module):
    """nn.MultiheadAttention's parameter set (packed in_proj, q|k|v rows) and init."""

    def __init__(self, embed_dim: int, num_heads: int):
        super().__init__()
        self.embed_dim = embed_dim
        self.num_heads = num_heads
        self.batch_first = True
        self.in_proj_weight = nn.Parameter(torch.empty(3 * embed_dim, embed_dim))
        self.in_proj_bias = nn.Parameter(torch.empty(3 * embed_dim))
        self.out_proj = nn.Linear(embed_dim, embed_dim)
        nn.init.xavier_uniform_(self.in_proj_weight)
        nn.init.zeros_(self.in_proj_bias)
        nn.init.zeros_(self.out_proj.bias)


class EncoderLayer(FerModule):
    """Post-norm transformer encoder layer (see module doc)."""

    def __init__(self, d_model: int, nhead: int, dim_feedforward: int = 2048, dropout: float = 0.1,
                 activation: str = "relu", layer_norm_eps: float = 1e-5):
        super().__init__()
        if d_model % nhead:
            raise ValueError("d_model must be divisible by nhead")
        self.self_attn = MultiheadAttentionParams(d_model, nhead)
        self.linear1 = nn.Linear(d_model, dim_feedforward)
        self.linear2 = nn.Linear(dim_feedforward, d_model)
        self.norm1 = nn.LayerNorm(d_model, eps=layer_norm_eps)
        self.norm2 = nn.LayerNorm(d_model, eps=layer_norm_eps)
        self.dropout_p = float(dropout)
        self.activation = activation
        self.norm_first = False

    def fer_params(self):
        a = self.self_attn
        return [a.in_proj_weight, a.in_proj_bias, a.out_proj.weight, a.out_proj.bias, self.linear1.weight,
                self.linear1.bias, self.linear2.weight, self.linear2.bias, self.norm1.weight, self.norm1.bias,
                self.norm2.weight, self.norm2.bias]

    def run_rows(self, t: torch.Tensor, B: int, N: int, save: bool) -> torch.Tensor:
        cfg = LayerCfg(B=B, N=N, H=self.self_attn.num_heads, act=self.activation,
                       dropout=self.dropout_p if self.training else 0.0, eps=self.norm1.eps, save=save)
        return PostNormLayerFn.apply(t, cfg, self.fer_flat(), *self.fer_params())

    def forward(self, src: torch.Tensor) -> torch.Tensor:
        t, B, N = _as_rows(src.to(self.compute_dtype()))
        save = self.need_grad(t, self.fer_params())
        return self.run_rows(t, B, N, save).view(B, N, -1)


class Encoder(FerModule):
    """nn.TransformerEncoder equivalent (`layers.{i}` deep copies of one prototype)."""

    def __init__(self, encoder_layer: EncoderLayer, num_layers: int):
        super().__init__()
        self.layers = nn.ModuleList([copy.deepcopy(encoder_layer) for _ in range(num_layers)])
        self.num_layers = num_layers

    def run_rows(self, t, B, N, save):
        for layer in self.layers:
            t = layer.run_rows(t, B, N, save)
        return t

    def forward(self, src: torch.Tensor) -> torch.Tensor:
        t, B, N = _as_rows(src.to(self.compute_dtype()))
        save = self.need_grad(t, list(self.parameters()))
        return self.run_rows(t, B, N, save).view(B, N, -1)


# ------------------------------------------------------------------ timm Block
class Attention(nn.Module):
    def __init__(self, dim: int, num_heads: int):
        super().__init__()
        self.num_heads = num_heads
        self.head_dim = dim // num_heads
        self.scale = self.head_dim ** -0.5
        self.qkv = nn.Linear(dim, dim * 3, bias=True)
        self.proj = nn.Linear(dim, dim)


class Mlp(nn.Module):
    def __init__(self, dim: int, hidden: int):
        super().__init__()
        self.fc1 = nn.Linear(dim, hidden)
        self.fc2 = nn.Linear(hidden, dim)


class Block(FerModule):
    """timm 1.0.17 `Block` (pre-norm, LN eps 1e-6, GELU, no dropout / layer-scale)."""

    def __init__(self, dim: int, num_heads: int, mlp_ratio: float = 4.0):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim, eps=1e-6)
        self.attn = Attention(dim, num_heads)
        self.norm2 = nn.LayerNorm(dim, eps=1e-6)
        self.mlp = Mlp(dim, int(dim * mlp_ratio))

    def fer_params(self):
        return [self.norm1.weight, self.norm1.bias, self.attn.qkv.weight, self.attn.qkv.bias, self.attn.proj.weight,
                self.attn.proj.bias, self.norm2.weight, self.norm2.bias, self.mlp.fc1.weight, self.mlp.fc1.bias,
                self.mlp.fc2.weight, self.mlp.fc2.bias]

    def run_rows(self, t, B, N, save):
        cfg = LayerCfg(B=B, N=N, H=self.attn.num_heads, act="gelu", dropout=0.0, eps=self.norm1.eps, save=save)
        return PreNormBlockFn.apply(t, cfg, self.fer_flat(), *self.fer_params())

    def forward(self, x):
        t, B, N = _as_rows(x.to(self.compute_dtype()))
        return self.run_rows(t, B, N, self.need_grad(t, self.fer_params())).view(B, N, -1)


def timm_vit_init_(module: nn.Module) -> None:
    """timm `init_weights_vit_timm`: trunc_normal(.02) Linear weights, zero biases."""
    for m in module.modules():
        if isinstance(m, nn.Linear):
            nn.init.trunc_normal_(m.weight, std=0.02)
            if m.bias is not None:
                nn.init.zeros_(m.bias)


class AdapterModule(FerModule):
    """x + alpha * fc2(GELU(fc1 x)) (`hybrid_latent_vit.py:249-265`)."""

    def __init__(self, embed_dim: int, adapter_dim: int):
        super().__init__()
        self.adapter = nn.Sequential(nn.Linear(embed_dim, adapter_dim), nn.GELU(), nn.Linear(adapter_dim, embed_dim))
        self.alpha = nn.Parameter(torch.ones(1) * 0.1)

    def fer_params(self):
        return [self.adapter[0].weight, self.adapter[0].bias, self.adapter[2].weight, self.adapter[2].bias,
                self.alpha]

    def run_rows(self, t, B, N, save):
        cfg = LayerCfg(B=B, N=N, H=1, save=save)
        return AdapterFn.apply(t, cfg, self.fer_flat(), *self.fer_params())

    def forward(self, x):
        t, B, N = _as_rows(x.to(self.compute_dtype()))
        return self.run_rows(t, B, N, self.need_grad(t, self.fer_params())).view(B, N, -1)


VIT_PRESETS = {
    "vit_tiny_patch16_224": dict(embed_dim=192, depth=12, num_heads=3),
    "vit_small_patch16_224": dict(embed_dim=384, depth=12, num_heads=6),
    "vit_base_patch16_224": dict(embed_dim=768, depth=12, num_heads=12),
}
