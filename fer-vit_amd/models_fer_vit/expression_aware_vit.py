"""ExpressionAwareViT (reference `models_fer_vit/expression_aware_vit.py:24-134`):
LatentDecomposer (fixed) -> HybridLatentViT.

Optional build-defined extension for BASELINE config 5 (not in the reference, which
never composes `modules/` with this model): `use_spe/use_lwn/use_lwn_residual/use_leam`
apply the LatentViTv2 prologue (SPE -> LWN -> LEAM, `latent_vit_v2.py:82-84`) to the
decomposer output before the ViT. All default to off (= reference behaviour).
"""
from typing import Literal, Optional

import torch
import torch.nn as nn

from fervit.module import FerModule
from modules import LEAM, LayerWiseNorm, SemanticPE
from modules._wplus import WplusSpec

from .hybrid_latent_vit import HybridLatentViT, create_hybrid_latent_vit
from .latent_decomposer import LatentDecomposer


class ExpressionAwareViT(FerModule):
    def __init__(self, decomposer: LatentDecomposer, vit_model: HybridLatentViT,
                 output_mode: Literal["expr_only", "id_only", "enhanced", "concat"] = "expr_only",
                 enhance_alpha: float = 2.0, decompose_mode: Literal["all_classes", "max_class"] = "all_classes",
                 use_spe: bool = False, use_lwn: bool = False, use_lwn_residual: bool = False,
                 use_leam: bool = False):
        super().__init__()
        self.decomposer = decomposer
        self.vit = vit_model
        self.output_mode = output_mode
        self.enhance_alpha = enhance_alpha
        self.decompose_mode = decompose_mode
        L, D = decomposer.seq_len, decomposer.latent_dim
        if (use_spe or use_lwn or use_leam) and output_mode == "concat":
            raise ValueError("the w+ prologue needs 18-token inputs; output_mode='concat' gives 36")
        self.use_spe, self.use_lwn, self.use_leam = use_spe, use_lwn, use_leam
        if use_spe:
            self.spe = SemanticPE(D, L)
        if use_lwn:
            self.lwn = LayerWiseNorm(L, D, use_residual=use_lwn_residual)
        if use_leam:
            self.leam = LEAM(L)
        print(f"\n[ExpressionAwareViT]\n  decompose_mode : {decompose_mode}\n  output_mode    : {output_mode}")
        if output_mode == "enhanced":
            print(f"  enhance_alpha  : {enhance_alpha}")

    @classmethod
    def from_config(cls, directions_path: str, model_size: str = "small", num_classes: int = 7,
                    use_pretrained: bool = True, freeze_transformer: bool = False,
                    freeze_stages: Optional[int] = None, use_adapter: bool = False, adapter_dim: int = 64,
                    output_mode="expr_only", enhance_alpha: float = 2.0, decompose_mode="all_classes",
                    **prologue) -> "ExpressionAwareViT":
        """`expression_aware_vit.py:53-107`."""
        decomposer = LatentDecomposer.from_file(directions_path)
        seq_len = decomposer.seq_len * (2 if output_mode == "concat" else 1)
        vit = create_hybrid_latent_vit(latent_dim=decomposer.latent_dim, seq_len=seq_len, model_size=model_size,
                                       num_classes=num_classes, use_pretrained=use_pretrained,
                                       freeze_transformer=freeze_transformer, freeze_stages=freeze_stages,
                                       use_adapter=use_adapter, adapter_dim=adapter_dim)
        return cls(decomposer, vit, output_mode, enhance_alpha, decompose_mode, **prologue)

    def forward(self, w_plus: torch.Tensor) -> torch.Tensor:
        flat = self.fer_flat()
        x = self.decomposer(w_plus, output_mode=self.output_mode, enhance_alpha=self.enhance_alpha,
                            decompose_mode=self.decompose_mode)
        if self.use_spe or self.use_lwn or self.use_leam:
            spec = WplusSpec(spe=getattr(self, "spe", None), lwn=getattr(self, "lwn", None),
                             leam=getattr(self, "leam", None))
            x = spec.run(x, flat, self.need_grad(None, spec.params()))
        return self.vit(x)

    def get_trainable_params(self):
        """`expression_aware_vit.py:124-126` (+ prologue params when enabled)."""
        P = [p for p in self.vit.parameters() if p.requires_grad]
        for name in ("spe", "lwn", "leam"):
            if hasattr(self, name):
                P += [p for p in getattr(self, name).parameters() if p.requires_grad]
        return P

    def print_info(self):
        total = sum(p.numel() for p in self.parameters())
        trainable = sum(p.numel() for p in self.parameters() if p.requires_grad)
        print(f"\n[ExpressionAwareViT] Parameters:\n  Total      : {total:,}")
        print(f"  Trainable  : {trainable:,} ({trainable / total * 100:.1f}%)")
        print("  Decomposer : fixed (SVM directions, not trained)")
