"""Host replica of the kernels' counter-based dropout hash (csrc/common.h fer_hash /
drop_keep), so tests can rebuild the exact keep-mask a kernel used."""
import numpy as np
import torch

_M32 = np.uint64(0xFFFFFFFF)


def _u32(x):
    return np.asarray(x, dtype=np.uint64) & _M32


def fer_hash(seed: int, pair: np.ndarray) -> np.ndarray:
    """csrc/common.h fer_hash: x = (pair ^ seed_lo) + seed_hi, then the lowbias32 finaliser."""
    pair = _u32(pair)
    s_lo, s_hi = np.uint64(seed & 0xFFFFFFFF), np.uint64((seed >> 32) & 0xFFFFFFFF)
    with np.errstate(over="ignore"):
        x = _u32((pair ^ s_lo) + s_hi)
        x ^= x >> np.uint64(16)
        x = _u32(x * np.uint64(0x7FEB352D))
        x ^= x >> np.uint64(15)
        x = _u32(x * np.uint64(0x846CA68B))
        x ^= x >> np.uint64(16)
    return x


def thresh(p: float) -> int:
    return max(1, min(65535, int(round(p * 65536.0))))


def keep_mask(seed: int, shape, p: float, base: int = 0) -> torch.Tensor:
    n = int(np.prod(shape))
    idx = np.arange(base, base + n, dtype=np.uint64) & _M32  # element indices are 32-bit
    h = fer_hash(seed, idx >> np.uint64(1))
    u = (h >> ((idx & np.uint64(1)) * np.uint64(16))) & np.uint64(0xFFFF)
    return torch.from_numpy((u >= np.uint64(thresh(p))).reshape(shape))


def keep_mask_torch(seed: int, shape, p: float, device="cuda") -> torch.Tensor:
    """keep_mask computed with int64 torch ops on `device` (large masks: a GPU test's attention
    dropout over B*H*N*N elements). 32-bit products are split into 16-bit halves so no int64
    product overflows."""
    n = int(np.prod(shape))
    m32 = 0xFFFFFFFF
    idx = torch.arange(n, dtype=torch.int64, device=device) & m32

    def mul32(x, c):
        return ((x * (c & 0xFFFF)) + (((x * (c >> 16)) & 0xFFFF) << 16)) & m32

    x = ((idx >> 1) ^ (seed & m32)) + ((seed >> 32) & m32)
    x &= m32
    x ^= x >> 16
    x = mul32(x, 0x7FEB352D)
    x ^= x >> 15
    x = mul32(x, 0x846CA68B)
    x ^= x >> 16
    u = (x >> ((idx & 1) * 16)) & 0xFFFF
    return (u >= thresh(p)).reshape(shape)
