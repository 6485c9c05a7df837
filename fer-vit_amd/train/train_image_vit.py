"""`train/train_image_vit.py` step functions (train_epoch 110-144, evaluate 147-178)."""
from __future__ import annotations

from .common import calculate_class_weights, run_evaluate, run_train_epoch, set_seed  # noqa: F401


def train_epoch(model, loader, optimizer, criterion, device, grad_clip=None):
    """zero_grad, forward, criterion, backward, optional clip_grad_norm_, step; metrics from the
    training logits. Returns (avg_loss, accuracy, f1_macro)."""
    return run_train_epoch(model, loader, optimizer, criterion, device, grad_clip=grad_clip)


def evaluate(model, loader, criterion, device):
    return run_evaluate(model, loader, criterion, device)
