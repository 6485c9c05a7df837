"""`train/train_expression_aware_vit.py` step functions (get_optimizer_groups 66-96 on
model.vit, train_epoch 99-122, evaluate 125-148)."""
from __future__ import annotations

from .common import (calculate_class_weights, layerwise_param_groups, run_evaluate, run_train_epoch,  # noqa: F401
                     set_seed)


def get_optimizer_groups(model, lr: float, weight_decay: float):
    return layerwise_param_groups(model.vit, lr, weight_decay)


def train_epoch(model, loader, optimizer, criterion, device):
    return run_train_epoch(model, loader, optimizer, criterion, device)


def evaluate(model, loader, criterion, device):
    return run_evaluate(model, loader, criterion, device)
