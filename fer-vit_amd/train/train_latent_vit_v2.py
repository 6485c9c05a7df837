"""`train/train_latent_vit_v2.py` step functions (train_epoch 107-149, evaluate 152-183):
args.mixup (default 1.0) and args.grad_clip (default 1.0, `:441`)."""
from __future__ import annotations

from .common import calculate_class_weights, run_evaluate, run_train_epoch, set_seed  # noqa: F401


def train_epoch(model, loader, optimizer, criterion, device, args):
    return run_train_epoch(model, loader, optimizer, criterion, device, mixup=float(args.mixup),
                           grad_clip=float(args.grad_clip) if args.grad_clip and args.grad_clip > 0 else None,
                           metric_forward=True)


def evaluate(model, loader, criterion, device):
    return run_evaluate(model, loader, criterion, device)
