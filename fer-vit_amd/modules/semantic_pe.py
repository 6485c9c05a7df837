"""SemanticPE — group (coarse/medium/fine) + per-layer learned embeddings added to the
w+ tokens (reference `modules/semantic_pe.py:11-48`); fused w+ prologue kernel."""
import torch
import torch.nn as nn

from fervit.module import FerModule

# layer -> group id (Coarse=0, Medium=1, Fine=2), `modules/semantic_pe.py:6-8`
_LAYER_GROUPS = [0] * 4 + [1] * 8 + [2] * 6


class SemanticPE(FerModule):
    def __init__(self, d_model: int = 512, num_layers: int = 18):
        super().__init__()
        self.group_embed = nn.Embedding(3, d_model)
        self.layer_embed = nn.Embedding(num_layers, d_model)
        self.register_buffer("groups", torch.tensor(_LAYER_GROUPS, dtype=torch.long))

    def forward(self, w_plus: torch.Tensor) -> torch.Tensor:
        from ._wplus import WplusSpec

        P = [self.group_embed.weight, self.layer_embed.weight]
        return WplusSpec(spe=self).run(w_plus, self.fer_flat(), self.need_grad(w_plus, P))
