"""Image ViT (reference `models_fer_vit/image_vit.py`): Conv2d patch embedding, CLS,
learned positions, post-norm GELU encoder, LayerNorm on CLS, linear head.

Constructor, attributes, init and state_dict keys follow the reference (`:11-205`);
the forward runs: im2col -> bf16 MFMA GEMM -> token assembly (PatchTokensFn), depth x
fused post-norm layer (PostNormLayerFn), fused LN+Linear head (HeadFn).
"""
import torch
import torch.nn as nn

from fervit.blocks import Encoder, EncoderLayer
from fervit.layers import HeadFn, LayerCfg, PatchTokensFn
from fervit.module import FerModule


class PatchEmbedding(FerModule):
    """`image_vit.py:11-44` — Conv2d(C, D, k=P, s=P) + flatten/transpose."""

    def __init__(self, img_size: int = 224, patch_size: int = 16, in_channels: int = 3, embed_dim: int = 768):
        super().__init__()
        self.img_size = img_size
        self.patch_size = patch_size
        self.n_patches = (img_size // patch_size) ** 2
        self.proj = nn.Conv2d(in_channels, embed_dim, kernel_size=patch_size, stride=patch_size)


class ImageViT(FerModule):
    def __init__(self, img_size: int = 224, patch_size: int = 16, in_channels: int = 3, embed_dim: int = 768,
                 depth: int = 12, heads: int = 12, mlp_dim: int = 3072, num_classes: int = 7,
                 dropout: float = 0.1):
        super().__init__()
        self.patch_size = patch_size
        self.n_patches = (img_size // patch_size) ** 2
        self.patch_embed = PatchEmbedding(img_size, patch_size, in_channels, embed_dim)
        self.cls_token = nn.Parameter(torch.randn(1, 1, embed_dim))
        self.pos_embed = nn.Parameter(torch.randn(1, self.n_patches + 1, embed_dim))
        self.dropout = nn.Dropout(dropout)
        layer = EncoderLayer(embed_dim, heads, mlp_dim, dropout, activation="gelu")
        self.transformer = Encoder(layer, num_layers=depth)
        self.norm = nn.LayerNorm(embed_dim)
        self.head = nn.Linear(embed_dim, num_classes)
        self._init_weights()

    def _init_weights(self):
        """`image_vit.py:119-135`."""
        nn.init.trunc_normal_(self.pos_embed, std=0.02)
        nn.init.trunc_normal_(self.cls_token, std=0.02)
        for module in self.modules():
            if isinstance(module, nn.Linear):
                nn.init.trunc_normal_(module.weight, std=0.02)
                if module.bias is not None:
                    nn.init.zeros_(module.bias)
            elif isinstance(module, nn.LayerNorm):
                nn.init.ones_(module.weight)
                nn.init.zeros_(module.bias)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """x: (B, C, H, W) -> logits (B, num_classes) fp32."""
        B = x.shape[0]
        flat = self.fer_flat()
        dt = self.compute_dtype()
        params = list(self.parameters())
        save = self.need_grad(None, params)
        N = self.n_patches + 1
        pe = self.patch_embed.proj
        cfg = LayerCfg(B=B, N=N, H=1, dropout=self.dropout.p if self.training else 0.0, save=save)
        t = PatchTokensFn.apply(x, cfg, flat, dt, self.patch_size, pe.weight, pe.bias, self.cls_token,
                                self.pos_embed)
        t = self.transformer.run_rows(t, B, N, save)
        hcfg = LayerCfg(B=B, N=N, H=1, eps=self.norm.eps, save=save)
        return HeadFn.apply(t, hcfg, flat, self.norm.weight, self.norm.bias, self.head.weight, self.head.bias)


def create_vit_small(num_classes: int = 7, img_size: int = 224) -> ImageViT:
    """ViT-Small/16 (`image_vit.py:169-179`)."""
    return ImageViT(img_size=img_size, patch_size=16, embed_dim=384, depth=12, heads=6, mlp_dim=1536,
                    num_classes=num_classes)


def create_vit_base(num_classes: int = 7, img_size: int = 224) -> ImageViT:
    """ViT-Base/16 (`image_vit.py:182-192`)."""
    return ImageViT(img_size=img_size, patch_size=16, embed_dim=768, depth=12, heads=12, mlp_dim=3072,
                    num_classes=num_classes)


def create_vit_tiny(num_classes: int = 7, img_size: int = 224) -> ImageViT:
    """ViT-Tiny/16 (`image_vit.py:195-205`)."""
    return ImageViT(img_size=img_size, patch_size=16, embed_dim=192, depth=12, heads=3, mlp_dim=768,
                    num_classes=num_classes)
