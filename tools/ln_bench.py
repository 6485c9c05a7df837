"""LayerNorm forward / backward at the ViT-B/16 bs=256 shape (M = 50432 rows, D = 768, bf16),
backward with the post-norm dropout copy and the dgamma/dbeta/dbias partials, as in the model.
HBM bytes: fwd 2 x M x D x 2; bwd 4 x M x D x 2 (dy, x in; dx, dx_drop out)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fer-vit_amd"))
import torch  # noqa: E402

from fervit import ops  # noqa: E402
from gemm_bench import timeit  # noqa: E402


def main():
    M, D = int(os.environ.get("LN_M", 256 * 197)), int(os.environ.get("LN_D", 768))
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(M, D, device="cuda", generator=g).to(torch.bfloat16)
    dy = torch.randn(M, D, device="cuda", generator=g).to(torch.bfloat16)
    w, b = torch.ones(D, device="cuda"), torch.zeros(D, device="cuda")
    mean, rstd = torch.empty(M, device="cuda"), torch.empty(M, device="cuda")
    y = ops.layernorm_fwd(x, w, b, 1e-5, mean=mean, rstd=rstd)
    dx, dxd = torch.empty_like(x), torch.empty_like(x)
    gg, gb, gd = (torch.zeros(D, device="cuda") for _ in range(3))
    tf = min(timeit(lambda: ops.layernorm_fwd(x, w, b, 1e-5, out=y, mean=mean, rstd=rstd)) for _ in range(3))
    tb = min(timeit(lambda: ops.layernorm_bwd(dy, x, mean, rstd, w, dx=dx, dx_drop=dxd, dropout=0.1, seed=3,
                                              dgamma=gg, dbeta=gb, dbias=gd)) for _ in range(3))
    print(f"ln fwd {tf * 1e3:6.1f} us ({2 * M * D * 2 / tf / 1e6:6.0f} GB/s)   "
          f"ln bwd {tb * 1e3:6.1f} us ({4 * M * D * 2 / tb / 1e6:6.0f} GB/s)", flush=True)


if __name__ == "__main__":
    main()
