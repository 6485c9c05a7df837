"""Fused softmax cross-entropy (nn.CrossEntropyLoss(label_smoothing, weight), mean
reduction; `train/train_image_vit.py:262-267`) on device, loss and dlogits in one launch."""
from __future__ import annotations

import torch

from . import ops


class _CEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, weight, ls):
        loss, dl = ops.cross_entropy(logits.contiguous().float(), labels.contiguous(), weight, ls)
        ctx.dl = dl
        return loss

    @staticmethod
    def backward(ctx, g):
        return ctx.dl * g, None, None, None


class CrossEntropyLoss(torch.nn.Module):
    def __init__(self, weight=None, label_smoothing: float = 0.0):
        super().__init__()
        self.weight = weight
        self.label_smoothing = float(label_smoothing)

    def forward(self, logits, labels):
        w = None if self.weight is None else self.weight.to(logits.device).float().contiguous()
        return _CEFn.apply(logits, labels.long(), w, self.label_smoothing)
