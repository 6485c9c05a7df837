"""Data-parallel launcher for the trainers (the reference trains on one device,
`train/train_image_vit.py:183`). One process per GPU started by torchrun
(`python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 ...`):

    rank, world, device = setup()
    model = wrap(model.to(device))                  # fervit.ddp.DistributedDataParallel (RCCL)
    loader = PackedLatentLoader(ds, 256, rank=rank, world_size=world, device=device)
    ...
    cleanup()

`wrap` broadcasts rank 0's parameters, then every backward all-reduces (AVG) the flat gradient
buffer in ~32 MB buckets on a side stream, overlapped with the rest of the backward.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from fervit.ddp import DistributedDataParallel


def setup(backend: str = "nccl"):
    """Initialise the process group from torchrun's environment; returns (rank, world, device).
    Without torchrun variables: single process (rank 0, world 1, cuda:0), no process group."""
    if "RANK" not in os.environ or "WORLD_SIZE" not in os.environ:
        return 0, 1, torch.device("cuda", 0)
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if not dist.is_initialized():
        if backend == "nccl":
            dist.init_process_group(backend, device_id=device)
        else:
            dist.init_process_group(backend)
    return dist.get_rank(), dist.get_world_size(), device


def wrap(model, bucket_cap_mb: float = 32.0):
    """DistributedDataParallel over the default group when one is initialised, else the model."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        return DistributedDataParallel(model, bucket_cap_mb=bucket_cap_mb)
    return model


def cleanup() -> None:
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
