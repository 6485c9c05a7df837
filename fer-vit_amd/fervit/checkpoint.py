"""Checkpoints in the reference's format.

`ExperimentLogger.save_checkpoint` (`utils/experiment_logger.py:121-145`) writes
{'epoch', 'model_state_dict', 'optimizer_state_dict', 'metrics', 'config', 'run_id'} with the
legacy (non-zip) serialization, and `eval/evaluate_model.py:30-132` rebuilds the model from
'config' and loads 'model_state_dict'. The models here keep the reference's state_dict keys,
and FusedAdamW emits torch.optim.AdamW-format state, so the same files move both ways:
build-trained checkpoints open in the reference's eval scripts, reference checkpoints resume here.
Loading uses `torch.load(weights_only=True)` with numpy scalars / dtypes allow-listed: the
reference stores `val_results` whose 'predictions' are numpy int64 values
(`train/train_latent_vit_v2.py:168,181`); nothing that executes code is allowed. Metrics written
here are converted to plain Python values first.
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
        "metrics": _plain(dict(metrics or {})),
        "config": dict(config or {}),
        "run_id": run_id,
    }
    torch.save(ckpt, path, _use_new_zipfile_serialization=False)
    return ckpt


def load_checkpoint(path: str, model: Optional[torch.nn.Module] = None,
                    optimizer: Optional[torch.optim.Optimizer] = None) -> Dict[str, Any]:
    """Load a checkpoint written by save_checkpoint or by the reference's ExperimentLogger
    ('model_state_dict' or the older 'model_state' key, `eval/evaluate_model.py:117-122`)."""
    ckpt = _safe_load(path)
    if model is not None:
        sd = ckpt.get("model_state_dict", ckpt.get("model_state"))
        if sd is None:
            raise KeyError("Model state dict not found in checkpoint")
        model.load_state_dict(sd)
    if optimizer is not None and ckpt.get("optimizer_state_dict"):
        optimizer.load_state_dict(ckpt["optimizer_state_dict"])
    return ckpt


def _safe_load(path: str):
    """torch.load(weights_only=True) with the numpy reconstructors allow-listed through the
    `safe_globals` context manager. Needs torch >= 2.5 (the reference pins 2.5.1,
    `environment.yml:113`; fervit.module's always_call forward hooks need >= 2.1 as well)."""
    ser = torch.serialization
    if not hasattr(ser, "safe_globals"):
        raise RuntimeError("fervit checkpoints need torch >= 2.5 (torch.serialization.safe_globals)")
    with ser.safe_globals(_numpy_safe_globals()):
        return torch.load(path, map_location="cpu", weights_only=True)


def _numpy_safe_globals():
    """numpy scalar / array reconstructors (numpy 2 and numpy 1.x module paths) and the dtype
    classes a pickled numpy value references. These only rebuild values; none runs user code
    (an object-dtype array would still need its element classes, which stay disallowed)."""
    import numpy as np

    try:  # numpy >= 2
        from numpy._core.multiarray import _reconstruct, scalar
    except ImportError:  # numpy 1.x (the reference allows numpy >= 1.21)
        from numpy.core.multiarray import _reconstruct, scalar
    try:
        import numpy.dtypes as ndt  # numpy >= 1.25
    except ImportError:
        ndt = None

    g = [scalar, (scalar, "numpy.core.multiarray.scalar"), _reconstruct,
         (_reconstruct, "numpy.core.multiarray._reconstruct"), np.ndarray, np.dtype]
    for name in ("Int8DType", "Int16DType", "Int32DType", "Int64DType", "UInt8DType", "UInt16DType", "UInt32DType",
                 "UInt64DType", "Float16DType", "Float32DType", "Float64DType", "BoolDType", "LongLongDType",
                 "LongDType"):
        if ndt is not None and hasattr(ndt, name):
            g.append(getattr(ndt, name))
    return g


def _plain(obj):
    """numpy scalars / arrays -> Python numbers / lists (checkpoint metrics)."""
    import numpy as np

    if isinstance(obj, np.generic):
        return obj.item()
    if isinstance(obj, np.ndarray):
        return obj.tolist()
    if isinstance(obj, dict):
        return {k: _plain(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_plain(v) for v in obj)
    return obj


def _to_cpu(obj):
    if torch.is_tensor(obj):
        return obj.detach().cpu()
    if isinstance(obj, dict):
        return {k: _to_cpu(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_cpu(v) for v in obj)
    return obj
