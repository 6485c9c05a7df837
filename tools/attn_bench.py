"""Attention microbenchmark at the ViT-B/16 bs=256 shape (B=256, N=197, H=12, dh=64, bf16):
forward and backward (dQ + dK/dV kernels) with and without probability dropout.
Algorithmic FLOP: fwd 4*N^2*dh per (b,h); bwd 8*N^2*dh (+ 2*N^2*dh S recompute per
orientation is not counted). HBM bytes: fwd reads q,k,v writes o; bwd reads q,k,v,o,dO
writes dq,dk,dv."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fer-vit_amd"))
import torch  # noqa: E402

from fervit import ops  # noqa: E402
from gemm_bench import timeit  # noqa: E402


def main():
    dev = "cuda"
    B, N, H, dh = int(os.environ.get("AB_B", 256)), 197, 12, 64
    D = H * dh
    M = B * N
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = torch.randn(M, 3 * D, device=dev, generator=g).to(torch.bfloat16)
    out = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    dout = torch.randn(M, D, device=dev, generator=g).to(torch.bfloat16)
    dqkv = torch.empty(M, 3 * D, device=dev, dtype=torch.bfloat16)
    fl_f = 4.0 * N * N * dh * B * H
    by_f = 2.0 * M * 4 * D
    by_b = 2.0 * M * 8 * D
    from fervit._lib import lib

    # forward kernels (fer_attention_set_fwd_kernel: 1 persistent, 2 occupancy form), interleaved
    for rep in range(2):
        for p in (0.1, 0.0):
            for fk in (1, 2):
                lib().fer_attention_set_fwd_kernel(fk)
                lse = ops.attention_saved(qkv, B, N, H, dh, dropout=p)
                tf = min(timeit(lambda: ops.attention_fwd(qkv, out, lse, B, N, H, dh, dropout=p, seed=5))
                         for _ in range(3))
                tb = min(timeit(lambda: ops.attention_bwd(qkv, out, dout, lse, dqkv, B, N, H, dh, dropout=p, seed=5))
                         for _ in range(3))
                print(f"p={p} fwd kernel {fk}: fwd {tf * 1e3:7.1f} us ({fl_f / tf / 1e9:6.1f} TF, "
                      f"{by_f / tf / 1e6:5.2f} GB/s)   bwd {tb * 1e3:7.1f} us ({2 * fl_f / tb / 1e9:6.1f} TF, "
                      f"{by_b / tb / 1e6:5.2f} GB/s)", flush=True)
    lib().fer_attention_set_fwd_kernel(0)  # back to automatic


if __name__ == "__main__":
    main()
