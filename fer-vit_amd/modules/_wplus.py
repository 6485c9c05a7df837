"""Shared spec for the fused w+ prologue kernel (SPE -> LWN -> LEAM).

Maps whichever of SemanticPE / LayerWiseNorm / LEAM are enabled onto the
contiguous [L][D] / [L] views of a flat parameter (or gradient) buffer that
`fer_wplus_fwd/bwd` expect (`latent_vit_v2.py:82-84` order).
"""
from __future__ import annotations

import torch

from fervit.layers import LayerCfg, WplusFn


class WplusSpec:
    def __init__(self, spe=None, lwn=None, leam=None):
        self.spe, self.lwn, self.leam = spe, lwn, leam
        self.groups = spe.groups if spe is not None else None

    def params(self):
        P = []
        if self.spe is not None:
            P += [self.spe.group_embed.weight, self.spe.layer_embed.weight]
        if self.lwn is not None:
            P += self.lwn._fer_local_order()
        if self.leam is not None:
            P += [self.leam.layer_weights]
        return P

    def _contig(self, flat, buf, params, rows, cols):
        o0 = flat.offsets[id(params[0])]
        for i, p in enumerate(params):
            if flat.offsets[id(p)] != o0 + i * cols:
                raise RuntimeError("fervit: LayerWiseNorm parameters are not contiguous in the flat buffer")
        return buf[o0:o0 + rows * cols].view(rows, cols)

    def views(self, buf, needs=None, flat=None):
        flat = flat or self.flat
        ok = (lambda p: True) if needs is None else (lambda p: needs.get(id(p), False))
        sg = sl = lw = lb = gate = lm = None
        if self.spe is not None:
            a, b = self.spe.group_embed.weight, self.spe.layer_embed.weight
            sg = flat.view(a, buf) if ok(a) else None
            sl = flat.view(b, buf) if ok(b) else None
        if self.lwn is not None:
            L = len(self.lwn.norms)
            D = self.lwn.norms[0].weight.numel()
            ws = [n.weight for n in self.lwn.norms]
            bs = [n.bias for n in self.lwn.norms]
            lw = self._contig(flat, buf, ws, L, D) if ok(ws[0]) else None
            lb = self._contig(flat, buf, bs, L, D) if ok(bs[0]) else None
            if self.lwn.use_residual:
                gate = flat.view(self.lwn.gate, buf) if ok(self.lwn.gate) else None
        if self.leam is not None:
            lm = flat.view(self.leam.layer_weights, buf) if ok(self.leam.layer_weights) else None
        if needs is None:
            # forward views must exist whenever the module is enabled
            if self.lwn is not None and self.lwn.use_residual and gate is None:
                raise RuntimeError("missing gate")
        return sg, sl, lw, lb, gate, lm

    def run(self, x: torch.Tensor, flat, training_save: bool) -> torch.Tensor:
        self.flat = flat
        B, L, D = x.shape
        if self.groups is not None and L > self.groups.numel():
            raise ValueError(f"SemanticPE supports at most {self.groups.numel()} w+ layers (got {L}); "
                             "the reference fails the same way (`modules/semantic_pe.py:44-47`)")
        cfg = LayerCfg(B=B, N=L, H=1, save=training_save)
        return WplusFn.apply(x, cfg, flat, self, *self.params())
