"""Host replica of the kernels' counter-based dropout hash (csrc/common.h fer_hash),
so tests can rebuild the exact keep-mask a kernel used."""
import numpy as np
import torch

_G = np.uint64(0x9E3779B97F4A7C15)
_M = np.uint64(0xD6E8FEB86659FD93)


def fer_hash(seed: int, idx: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = idx.astype(np.uint64) + np.uint64(seed & 0xFFFFFFFFFFFFFFFF) * _G
        z ^= z >> np.uint64(32)
        z *= _M
        z ^= z >> np.uint64(32)
        z *= _M
        z ^= z >> np.uint64(32)
    return (z & np.uint64(0xFFFFFFFF)).astype(np.uint64)


def keep_mask(seed: int, shape, p: float, base: int = 0) -> torch.Tensor:
    thr = min(int(p * 4294967296.0), 4294967295)
    n = int(np.prod(shape))
    idx = np.arange(base, base + n, dtype=np.uint64)
    k = fer_hash(seed, idx) >= np.uint64(thr)
    return torch.from_numpy(k.reshape(shape))
