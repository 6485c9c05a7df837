"""HybridLatentViT (reference `models_fer_vit/hybrid_latent_vit.py:18-343`): w+ tokens ->
Linear -> ViT blocks (timm `vit_{tiny,small,base}_patch16_224` geometry) [+ per-block
Adapter] -> LN / Dropout / Linear head.

timm is not a dependency here: the blocks are fervit `Block`s with timm's parameter
names (`transformer.{i}.norm1/attn.qkv/attn.proj/norm2/mlp.fc1/mlp.fc2`) and timm's
random init. `use_pretrained=True` loads a local timm checkpoint from
$FERVIT_PRETRAINED_DIR/<model_name>.{safetensors,pth} (no network access); the
positional embedding is then interpolated 196 -> seq_len exactly as the reference does
(`:118-156`).
"""
import os
from typing import Literal, Optional

import torch
import torch.nn as nn

from fervit.blocks import VIT_PRESETS, AdapterModule, Block, timm_vit_init_
from fervit.layers import HeadFn, LatentTokensFn, LayerCfg
from fervit.module import FerModule


def _load_pretrained(name: str):
    d = os.environ.get("FERVIT_PRETRAINED_DIR")
    if d:
        for ext in (".safetensors", ".pth", ".bin"):
            p = os.path.join(d, name + ext)
            if os.path.exists(p):
                if ext == ".safetensors":
                    from safetensors.torch import load_file

                    return load_file(p)
                return torch.load(p, map_location="cpu", weights_only=True)
    raise RuntimeError(f"pretrained weights for {name} are not available offline: set use_pretrained=False or "
                       f"place {name}.safetensors/.pth (timm format) under $FERVIT_PRETRAINED_DIR")


class _PretrainedViT(nn.Module):
    """Stand-in for timm.create_model(name, num_classes=0): cls_token, pos_embed, blocks."""

    def __init__(self, name: str, pretrained: bool):
        super().__init__()
        cfg = VIT_PRESETS[name]
        D = cfg["embed_dim"]
        self.embed_dim = D
        self.cls_token = nn.Parameter(torch.zeros(1, 1, D))
        self.pos_embed = nn.Parameter(torch.zeros(1, 197, D))
        self.blocks = nn.Sequential(*[Block(D, cfg["num_heads"]) for _ in range(cfg["depth"])])
        nn.init.trunc_normal_(self.pos_embed, std=0.02)
        nn.init.normal_(self.cls_token, std=1e-6)
        timm_vit_init_(self.blocks)
        if pretrained:
            sd = _load_pretrained(name)
            own = {k: v for k, v in sd.items() if k.startswith("blocks.") or k in ("cls_token", "pos_embed")}
            self.load_state_dict(own, strict=False)


class HybridLatentViT(FerModule):
    def __init__(self, latent_dim: int = 512, seq_len: int = 18, pretrained_model_name: str = "vit_small_patch16_224",
                 num_classes: int = 7, use_pretrained: bool = True, freeze_transformer: bool = False,
                 freeze_stages: Optional[int] = None, adapter_dim: Optional[int] = None):
        super().__init__()
        if pretrained_model_name not in VIT_PRESETS:
            raise ValueError(f"unsupported backbone {pretrained_model_name}; choose one of {list(VIT_PRESETS)}")
        self.latent_dim = latent_dim
        self.seq_len = seq_len
        self.num_classes = num_classes
        self.pretrained_model_name = pretrained_model_name
        self.use_adapter = adapter_dim is not None
        print(f"\n{'=' * 60}\nLoading pretrained model: {pretrained_model_name}\n{'=' * 60}")
        pretrained_vit = _PretrainedViT(pretrained_model_name, use_pretrained)
        self.embed_dim = pretrained_vit.embed_dim
        print(f"Pretrained model embedding dimension: {self.embed_dim}")
        self.input_proj = nn.Linear(latent_dim, self.embed_dim)
        self.cls_token = nn.Parameter(pretrained_vit.cls_token.data.clone())
        self.pos_embed = self._init_position_embedding(pretrained_vit, seq_len)
        self.transformer = pretrained_vit.blocks
        print(f"Extracted {len(self.transformer)} transformer blocks from pretrained model")
        if self.use_adapter:
            print(f"Using adapter layers with dim={adapter_dim}")
            self.adapters = nn.ModuleList([AdapterModule(self.embed_dim, adapter_dim) for _ in self.transformer])
        if freeze_transformer:
            self._freeze_transformer()
        elif freeze_stages is not None:
            self._freeze_stages(freeze_stages)
        self.head = nn.Sequential(nn.LayerNorm(self.embed_dim), nn.Dropout(0.1),
                                  nn.Linear(self.embed_dim, num_classes))
        self._print_model_info()

    def _init_position_embedding(self, pretrained_vit, seq_len):
        """`hybrid_latent_vit.py:118-156`: keep, or 1-D linear interpolation of the patch part."""
        pos = pretrained_vit.pos_embed
        n = pos.size(1) - 1
        if seq_len == n:
            return nn.Parameter(pos.data.clone())
        print(f"Interpolating position embeddings: {n} → {seq_len}")
        cls_pos = pos[:, 0:1, :]
        patch = pos[:, 1:, :].permute(0, 2, 1)
        patch = nn.functional.interpolate(patch, size=seq_len, mode="linear", align_corners=False).permute(0, 2, 1)
        return nn.Parameter(torch.cat([cls_pos, patch], dim=1).detach().clone())

    def _freeze_transformer(self):
        for p in self.transformer.parameters():
            p.requires_grad = False
        print("Transformer frozen")

    def _freeze_stages(self, n_stages: int):
        n_stages = min(n_stages, len(self.transformer))
        for i in range(n_stages):
            for p in self.transformer[i].parameters():
                p.requires_grad = False
        print(f"Frozen first {n_stages}/{len(self.transformer)} transformer blocks")

    def _print_model_info(self):
        total = sum(p.numel() for p in self.parameters())
        trainable = sum(p.numel() for p in self.parameters() if p.requires_grad)
        print(f"\n{'=' * 60}\nModel Information:\n{'=' * 60}")
        print(f"  Input: Latent codes ({self.seq_len}, {self.latent_dim})")
        print(f"  Transformer embedding dim: {self.embed_dim}")
        print(f"  Number of transformer blocks: {len(self.transformer)}")
        print(f"  Output classes: {self.num_classes}")
        print(f"  Adapter: {'Yes' if self.use_adapter else 'No'}")
        print(f"\nParameters:\n  Total: {total:,}")
        print(f"  Trainable: {trainable:,} ({trainable / total * 100:.1f}%)")
        print(f"  Frozen: {total - trainable:,} ({(total - trainable) / total * 100:.1f}%)\n{'=' * 60}\n")

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """x: (B, seq_len, latent_dim) -> logits (B, num_classes)."""
        B, L, _ = x.shape
        flat = self.fer_flat()
        save = self.need_grad(x, list(self.parameters()))
        N = L + 1
        cfg = LayerCfg(B=B, N=N, H=1, save=save)
        t = LatentTokensFn.apply(x, cfg, flat, self.compute_dtype(), self.input_proj.weight, self.input_proj.bias,
                                 self.cls_token, self.pos_embed)
        for i, block in enumerate(self.transformer):
            t = block.run_rows(t, B, N, save)
            if self.use_adapter:
                t = self.adapters[i].run_rows(t, B, N, save)
        ln, drop, lin = self.head[0], self.head[1], self.head[2]
        hcfg = LayerCfg(B=B, N=N, H=1, eps=ln.eps, dropout=drop.p if self.training else 0.0, save=save)
        return HeadFn.apply(t, hcfg, flat, ln.weight, ln.bias, lin.weight, lin.bias)

    def unfreeze_all(self):
        for p in self.parameters():
            p.requires_grad = True
        print("All parameters unfrozen")
        self._print_model_info()


def create_hybrid_latent_vit(latent_dim: int = 512, seq_len: int = 18,
                             model_size: Literal["tiny", "small", "base"] = "small", num_classes: int = 7,
                             use_pretrained: bool = True, freeze_transformer: bool = False,
                             freeze_stages: Optional[int] = None, use_adapter: bool = False,
                             adapter_dim: int = 64) -> HybridLatentViT:
    """`hybrid_latent_vit.py:268-310`."""
    names = {"tiny": "vit_tiny_patch16_224", "small": "vit_small_patch16_224", "base": "vit_base_patch16_224"}
    return HybridLatentViT(latent_dim=latent_dim, seq_len=seq_len,
                           pretrained_model_name=names.get(model_size, "vit_small_patch16_224"),
                           num_classes=num_classes, use_pretrained=use_pretrained,
                           freeze_transformer=freeze_transformer, freeze_stages=freeze_stages,
                           adapter_dim=adapter_dim if use_adapter else None)


# `hybrid_latent_vit.py:314-343`
RECOMMENDED_STRATEGIES = {
    "full_finetune": {"freeze_transformer": False, "freeze_stages": None, "use_adapter": False, "lr": 1e-4,
                      "description": "全パラメータを学習（最高精度、学習時間長）"},
    "partial_freeze": {"freeze_transformer": False, "freeze_stages": 6, "use_adapter": False, "lr": 3e-4,
                       "description": "下位層凍結（バランス）"},
    "adapter": {"freeze_transformer": True, "freeze_stages": None, "use_adapter": True, "lr": 1e-3,
                "description": "アダプター層のみ学習（最速、メモリ効率的）"},
    "linear_probe": {"freeze_transformer": True, "freeze_stages": None, "use_adapter": False, "lr": 1e-3,
                     "description": "分類ヘッドのみ学習（ベースライン）"},
}
