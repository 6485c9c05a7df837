"""LEAM — Layer-wise Expression Attention Mask (reference `modules/leam.py:5-44`).

y = w+ * sigmoid(layer_weights)[l]; runs in the fused w+ prologue kernel.
"""
import torch
import torch.nn as nn

from fervit.module import FerModule


class LEAM(FerModule):
    def __init__(self, num_layers: int = 18, init_coarse: float = 0.5, init_fine: float = 0.5):
        super().__init__()
        init = torch.ones(num_layers)
        init[:4] = init_coarse
        init[12:] = init_fine
        self.layer_weights = nn.Parameter(init)

    def forward(self, w_plus: torch.Tensor) -> torch.Tensor:
        from ._wplus import WplusSpec

        return WplusSpec(leam=self).run(w_plus, self.fer_flat(), self.need_grad(w_plus, [self.layer_weights]))

    def get_weights(self) -> torch.Tensor:
        """Visualisation helper (`modules/leam.py:42-44`)."""
        return torch.sigmoid(self.layer_weights).detach().cpu()
