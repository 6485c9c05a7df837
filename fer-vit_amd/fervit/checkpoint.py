"""Checkpoints in the reference's format.

`ExperimentLogger.save_checkpoint` (`utils/experiment_logger.py:121-145`) writes
{'epoch', 'model_state_dict', 'optimizer_state_dict', 'metrics', 'config', 'run_id'} with the
legacy (non-zip) serialization, and `eval/evaluate_model.py:30-132` rebuilds the model from
'config' and loads 'model_state_dict'. The models here keep the reference's state_dict keys,
and FusedAdamW emits torch.optim.AdamW-format state, so the same files move both ways:
build-trained checkpoints open in the reference's eval scripts, reference checkpoints resume here.
Loading uses `torch.load(weights_only=True)`: the dict holds only tensors and plain values.
"""
from __future__ import annotations

from typing import Any, Dict, Optional

import torch


def save_checkpoint(path: str, model: torch.nn.Module, optimizer: Optional[torch.optim.Optimizer], epoch: int,
                    metrics: Optional[Dict[str, float]] = None, config: Optional[Dict[str, Any]] = None,
                    run_id: Optional[str] = None) -> Dict[str, Any]:
    ckpt = {
        "epoch": epoch,
        "model_state_dict": {k: v.detach().cpu() for k, v in model.state_dict().items()},
        "optimizer_state_dict": _to_cpu(optimizer.state_dict()) if optimizer is not None else {},
        "metrics": dict(metrics or {}),
        "config": dict(config or {}),
        "run_id": run_id,
    }
    torch.save(ckpt, path, _use_new_zipfile_serialization=False)
    return ckpt


def load_checkpoint(path: str, model: Optional[torch.nn.Module] = None,
                    optimizer: Optional[torch.optim.Optimizer] = None) -> Dict[str, Any]:
    """Load a checkpoint written by save_checkpoint or by the reference's ExperimentLogger
    ('model_state_dict' or the older 'model_state' key, `eval/evaluate_model.py:117-122`)."""
    ckpt = torch.load(path, map_location="cpu", weights_only=True)
    if model is not None:
        sd = ckpt.get("model_state_dict", ckpt.get("model_state"))
        if sd is None:
            raise KeyError("Model state dict not found in checkpoint")
        model.load_state_dict(sd)
    if optimizer is not None and ckpt.get("optimizer_state_dict"):
        optimizer.load_state_dict(ckpt["optimizer_state_dict"])
    return ckpt


def _to_cpu(obj):
    if torch.is_tensor(obj):
        return obj.detach().cpu()
    if isinstance(obj, dict):
        return {k: _to_cpu(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_cpu(v) for v in obj)
    return obj
