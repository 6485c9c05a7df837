"""LayerWiseNorm — an independent LayerNorm per w+ layer, optional residual gate
out = w+ + sigmoid(gate) * (LN_l(w+) - w+) (reference `modules/layer_wise_norm.py:5-50`).
Parameters keep the reference's `norms.{l}.weight/bias`, `gate` names; in the flat
buffer the weights (then the biases) are laid out contiguously as one [L][D] table so
the fused prologue kernel reads them directly."""
import torch
import torch.nn as nn

from fervit.module import FerModule


class LayerWiseNorm(FerModule):
    def __init__(self, num_layers: int = 18, d_model: int = 512, use_residual: bool = False):
        super().__init__()
        self.norms = nn.ModuleList([nn.LayerNorm(d_model) for _ in range(num_layers)])
        self.use_residual = use_residual
        if use_residual:
            self.gate = nn.Parameter(torch.full((num_layers,), -5.0))

    def _fer_local_order(self):
        P = [n.weight for n in self.norms] + [n.bias for n in self.norms]
        if self.use_residual:
            P.append(self.gate)
        return P

    def forward(self, w_plus: torch.Tensor) -> torch.Tensor:
        from ._wplus import WplusSpec

        return WplusSpec(lwn=self).run(w_plus, self.fer_flat(), self.need_grad(w_plus, self._fer_local_order()))
