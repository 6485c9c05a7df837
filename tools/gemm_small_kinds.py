"""Fused-epilogue GEMMs at the w+ latent shapes of the hybrid / expression configs (bs=256 x 19
tokens = 4864 rows, timm-B/16 widths D=768, F=3072): the 128^2-tile kernel with each epilogue
kind the layers use (bias store, GELU gate + dropout, bias + dropout + residual, gate multiply)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fer-vit_amd"))
import torch  # noqa: E402

from fervit import ops  # noqa: E402
from gemm_bench import timeit  # noqa: E402


def main():
    M, D, F = 256 * 19, 768, 3072
    g = torch.Generator(device="cuda").manual_seed(0)
    r = lambda *s: torch.randn(*s, device="cuda", generator=g).to(torch.bfloat16)
    x, h = r(M, D), r(M, F)
    wqkv, wo, w1, w2, w2t = r(3 * D, D), r(D, D), r(F, D), r(D, F), r(F, D)
    w1t, wqt = r(D, F), r(D, 3 * D)
    dq = r(M, 3 * D)
    bq, bo, b1, b2 = (torch.zeros(n, device="cuda") for n in (3 * D, D, F, D))
    gate = torch.empty(M, F, device="cuda", dtype=torch.bfloat16)
    cs = torch.zeros(F, device="cuda")
    cases = {
        "qkv fwd (store)": (lambda: ops.linear_fwd(x, wqkv, bq), 2 * M * 3 * D * D),
        "out fwd (res+drop)": (lambda: ops.linear_fwd(x, wo, bo, res=x, dropout=0.1, seed=3, drop_ld=D), 2 * M * D * D),
        "fc1 fwd (gate)": (lambda: ops.linear_fwd(x, w1, b1, pre=gate, pre_gate=True, act="gelu", dropout=0.1, seed=5,
                                                  drop_ld=F), 2 * M * F * D),
        "fc2 fwd (res+drop)": (lambda: ops.linear_fwd(h, w2, b2, res=x, dropout=0.1, seed=7, drop_ld=D), 2 * M * F * D),
        "fc2 dgrad (mul+cs)": (lambda: ops.linear_fwd(x, w2t, aux=gate, aux_act="mul", colsum=cs), 2 * M * F * D),
        # the frozen trunk's input gradients (timm pre-norm block: no epilogue)
        "fc1 dgrad (store)": (lambda: ops.linear_fwd(h, w1t), 2 * M * F * D),
        "proj dgrad (store)": (lambda: ops.linear_fwd(x, wo), 2 * M * D * D),
        "qkv dgrad (store)": (lambda: ops.linear_fwd(dq, wqt), 2 * M * 3 * D * D),
    }
    tot = 0.0
    for k, (fn, fl) in cases.items():
        t = min(timeit(fn) for _ in range(3))
        tot += t
        print(f"{k:20s} {t * 1e3:7.1f} us {fl / t / 1e9:6.1f} TF", flush=True)
    print(f"sum {tot * 1e3:.1f} us", flush=True)


if __name__ == "__main__":
    main()
