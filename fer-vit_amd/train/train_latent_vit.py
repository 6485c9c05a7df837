"""`train/train_latent_vit.py` step functions (train_epoch 108-149, evaluate 152-183). The
reference reads the mixup alpha from its module-level `args` (CLI default 1.0, `:407`); here it
is the `mixup` argument."""
from __future__ import annotations

from .common import calculate_class_weights, run_evaluate, run_train_epoch, set_seed  # noqa: F401


def train_epoch(model, loader, optimizer, criterion, device, mixup: float = 1.0):
    """Mixup step + a second no-grad forward on the unmixed batch for the metrics."""
    return run_train_epoch(model, loader, optimizer, criterion, device, mixup=mixup, metric_forward=True)


def evaluate(model, loader, criterion, device):
    return run_evaluate(model, loader, criterion, device)
