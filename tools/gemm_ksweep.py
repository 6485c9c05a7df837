"""Per-tile fixed cost vs per-K-step cost: time Y = X W^T at M=50432, N=3072 for several K
(linear fit t = a + b*K per round of tiles)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fer-vit_amd"))
import torch  # noqa: E402

from fervit import ops  # noqa: E402
from gemm_bench import timeit  # noqa: E402

dev = "cuda"
M, N = 50432, int(os.environ.get("KS_N", "3072"))
g = torch.Generator(device=dev).manual_seed(0)
res = []
for K in (64, 128, 256, 512, 768, 1536, 3072):
    x = torch.randn(M, K, device=dev, generator=g, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=dev, generator=g, dtype=torch.bfloat16) * 0.03
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    t = min(timeit(lambda: ops.linear_fwd(x, w, out=out)) for _ in range(3))
    tr = min(timeit(lambda: torch.matmul(x, w.t(), out=out)) for _ in range(3))
    fl = 2 * M * N * K
    res.append((K, t))
    print(f"[cfg {os.environ.get('FERVIT_GEMM_CFG', 'auto')}] N={N} K={K:5d} ours {t*1e3:8.1f} us {fl/t/1e9:7.1f} TF   "
          f"hipBLASLt {tr*1e3:8.1f} us {fl/tr/1e9:7.1f} TF", flush=True)
