"""Shared pieces of the training steps (`train/train_*.py` train_epoch / evaluate, SURVEY §8
a16), re-done without per-step host synchronisation: the reference calls `loss.item()` and
`preds.cpu()` every step (`train/train_image_vit.py:132-137`), which stalls the stream; here
the loss sum, predictions and labels stay on the device and cross to the host once per epoch,
where accuracy / F1 are computed by the same sklearn calls as the reference.
"""
from __future__ import annotations

import random
from collections import Counter
from typing import Dict, List, Optional

import numpy as np
import torch

from fervit.optim import FusedAdamW, clip_grad_norm_ as fused_clip_grad_norm_


def set_seed(seed: int = 42) -> None:
    """`train/train_image_vit.py:30-41`."""
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    torch.cuda.manual_seed_all(seed)


def calculate_class_weights(dataset) -> torch.Tensor:
    """total / (num_classes * count) per class (`train/train_image_vit.py:82-107`); uses the
    packed shard's label table when available instead of loading every sample."""
    if hasattr(dataset, "get_class_counts") and not hasattr(dataset, "indices"):
        counts = Counter(dataset.get_class_counts())
        total = sum(counts.values())
    else:
        base = getattr(dataset, "dataset", dataset)
        idx = getattr(dataset, "indices", range(len(dataset)))
        labels = [int(base[i][1]) for i in idx]
        counts, total = Counter(labels), len(labels)
    nc = len(counts)
    return torch.FloatTensor([total / (nc * counts[i]) if i in counts else 1.0 for i in range(nc)])


def _core(model):
    return getattr(model, "module", model)  # DistributedDataParallel wrapper


def clip_gradients(model, optimizer, max_norm: float) -> None:
    """clip_grad_norm_ without a host round trip: on the flat gradient buffer (coefficient
    consumed by FusedAdamW) or torch's for other optimizers."""
    if isinstance(optimizer, FusedAdamW) and hasattr(_core(model), "fer_flat"):
        fused_clip_grad_norm_(_core(model), max_norm, optimizer=optimizer)
    else:
        torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm)


class EpochStats:
    """Device-side loss sum and prediction / label record of one epoch."""

    def __init__(self, device):
        self.loss = torch.zeros((), dtype=torch.float64, device=device)
        self.preds: List[torch.Tensor] = []
        self.labels: List[torch.Tensor] = []

    def add(self, loss: torch.Tensor, n: int, logits: torch.Tensor, labels: torch.Tensor) -> None:
        self.loss += loss.detach().double() * n
        self.preds.append(logits.detach().argmax(dim=1))
        self.labels.append(labels.detach())

    def finish(self, n_samples: int) -> Dict:
        from sklearn.metrics import accuracy_score, f1_score

        preds = torch.cat(self.preds).cpu().numpy() if self.preds else np.zeros(0, np.int64)
        labels = torch.cat(self.labels).cpu().numpy() if self.labels else np.zeros(0, np.int64)
        return {
            "loss": float(self.loss.item()) / max(n_samples, 1),
            "accuracy": accuracy_score(labels, preds),
            "f1_macro": f1_score(labels, preds, average="macro"),
            "f1_weighted": f1_score(labels, preds, average="weighted"),
            "predictions": preds.tolist(),
            "labels": labels.tolist(),
        }


def run_train_epoch(model, loader, optimizer, criterion, device, mixup: Optional[float] = None, grad_clip=None,
                    metric_forward: bool = False):
    """One epoch of the reference step: [mixup, when `mixup` is not None (the latent trainers:
    lam ~ Beta(a, a) from numpy's global RNG, or 1 for a <= 0, and a CPU randperm every step,
    as `train/train_latent_vit_v2.py:118-125`)], zero_grad, forward,
    criterion (mixed as lam*CE(y) + (1-lam)*CE(y[perm])), backward, [clip], step; metrics from
    the training logits, or (metric_forward) from a second no-grad forward on the unmixed
    batch (`train_latent_vit_v2.py:137-141`). Returns (avg_loss, accuracy, f1_macro)."""
    model.train()
    stats = EpochStats(device)
    n = 0
    for x, y in loader:
        x = x.to(device, non_blocking=True)
        y = y.to(device, non_blocking=True)
        b = x.size(0)
        n += b
        if mixup is not None:
            lam = np.random.beta(mixup, mixup) if mixup > 0 else 1.0
            index = torch.randperm(b).to(device)
            xin = lam * x + (1 - lam) * x[index]
        else:
            lam, index, xin = 1.0, None, x
        optimizer.zero_grad()
        logits = model(xin)
        if index is not None:
            loss = lam * criterion(logits, y) + (1 - lam) * criterion(logits, y[index])
        else:
            loss = criterion(logits, y)
        loss.backward()
        if grad_clip is not None and grad_clip > 0:
            clip_gradients(model, optimizer, grad_clip)
        optimizer.step()
        if metric_forward:
            with torch.no_grad():
                stats.add(loss, b, model(x), y)
        else:
            stats.add(loss, b, logits, y)
    ds = getattr(loader, "dataset", None)
    r = stats.finish(len(ds) if ds is not None else n)
    return r["loss"], r["accuracy"], r["f1_macro"]


@torch.no_grad()
def run_evaluate(model, loader, criterion, device) -> Dict:
    """`train/train_image_vit.py:147-178` (same keys), one host transfer per call."""
    model.eval()
    stats = EpochStats(device)
    n = 0
    for x, y in loader:
        x = x.to(device, non_blocking=True)
        y = y.to(device, non_blocking=True)
        logits = model(x)
        stats.add(criterion(logits, y), x.size(0), logits, y)
        n += x.size(0)
    ds = getattr(loader, "dataset", None)
    return stats.finish(len(ds) if ds is not None else n)


def layerwise_param_groups(vit, lr: float, weight_decay: float, log=print) -> list:
    """`train/train_hybrid_latent_vit.py:63-117` / `train_expression_aware_vit.py:66-96`:
    input_proj, adapters and head at 10x lr, transformer at lr (trainable only), pos/cls at 5x
    without weight decay."""
    groups = []
    p = list(vit.input_proj.parameters())
    if p:
        groups.append({"params": p, "lr": lr * 10, "weight_decay": weight_decay})
        log(f"Input projection: lr={lr * 10:.2e}")
    p = [q for q in vit.transformer.parameters() if q.requires_grad]
    if p:
        groups.append({"params": p, "lr": lr, "weight_decay": weight_decay})
        log(f"Transformer: lr={lr:.2e}, params={len(p)}")
    if getattr(vit, "use_adapter", False):
        p = [q for q in vit.adapters.parameters() if q.requires_grad]
        if p:
            groups.append({"params": p, "lr": lr * 10, "weight_decay": weight_decay})
            log(f"Adapters: lr={lr * 10:.2e}")
    p = list(vit.head.parameters())
    if p:
        groups.append({"params": p, "lr": lr * 10, "weight_decay": weight_decay})
        log(f"Head: lr={lr * 10:.2e}")
    groups.append({"params": [vit.pos_embed, vit.cls_token], "lr": lr * 5, "weight_decay": 0})
    log(f"Position/CLS: lr={lr * 5:.2e}")
    return groups
