"""One ViT-B/16 bs=256 GEMM launch with its real epilogue, run a few times (PMC / trace target).

    GEMM_CASE=gate|res_fc2|res_out|res_fc1d|mul|store_qkv|store_outd|plain_fc1|wgrad python tools/gemm_case.py

The calls are the ones fervit/layers.py PostNormLayerFn makes (random N(0,1) data)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fer-vit_amd"))
import torch  # noqa: E402

from fervit import ops  # noqa: E402

M, D, F = 256 * 197, 768, 3072


def make_cases(dev="cuda"):
    g = torch.Generator(device=dev).manual_seed(0)
    r = lambda *s: torch.randn(*s, device=dev, generator=g, dtype=torch.bfloat16)  # noqa: E731
    x, h, dF = r(M, D), r(M, F), r(M, F)
    w1, w2, wq, wo = r(F, D) * 0.03, r(D, F) * 0.03, r(3 * D, D) * 0.03, r(D, D) * 0.03
    w1t, w2t, wqt = w1.t().contiguous(), w2.t().contiguous(), wq.t().contiguous()
    b1, bD, b3 = torch.zeros(F, device=dev), torch.zeros(D, device=dev), torch.zeros(3 * D, device=dev)
    gate = torch.empty(M, F, device=dev, dtype=torch.bfloat16)
    out_f = torch.empty(M, F, device=dev, dtype=torch.bfloat16)
    out_d = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    out_3 = torch.empty(M, 3 * D, device=dev, dtype=torch.bfloat16)
    dq = r(M, 3 * D)
    cs = torch.zeros(F, device=dev)
    gw = torch.zeros(F, D, device=dev)
    gwo, gwq = torch.zeros(D, D, device=dev), torch.zeros(3 * D, D, device=dev)
    p = 0.1
    return {
        # name: (launch, flop)
        "gate": (lambda: ops.linear_fwd(x, w1, b1, out=out_f, pre=gate, pre_gate=True, act="gelu", dropout=p,
                                        seed=7, drop_ld=F), 2 * M * F * D),
        "res_fc2": (lambda: ops.linear_fwd(h, w2, bD, out=out_d, res=x, dropout=p, seed=8, drop_ld=D), 2 * M * F * D),
        "res_out": (lambda: ops.linear_fwd(x, wo, bD, out=out_d, res=x, dropout=p, seed=9, drop_ld=D), 2 * M * D * D),
        "res_fc1d": (lambda: ops.linear_fwd(dF, w1t, out=out_d, res=x), 2 * M * F * D),
        "res_qkvd": (lambda: ops.linear_fwd(dq, wqt, out=out_d, res=x), 2 * M * 3 * D * D),
        "mul": (lambda: ops.linear_fwd(x, w2t, out=out_f, aux=gate, aux_act="mul", colsum=cs), 2 * M * F * D),
        "store_qkv": (lambda: ops.linear_fwd(x, wq, b3, out=out_3), 2 * M * 3 * D * D),
        "store_outd": (lambda: ops.linear_fwd(x, wo, out=out_d), 2 * M * D * D),
        "plain_fc1": (lambda: ops.linear_fwd(x, w1, out=out_f), 2 * M * F * D),
        "wgrad": (lambda: ops.linear_wgrad(dF, x, gw), 2 * M * F * D),
        "wgrad_out": (lambda: ops.linear_wgrad(x, x, gwo), 2 * M * D * D),
        "wgrad_qkv": (lambda: ops.linear_wgrad(dq, x, gwq), 2 * M * 3 * D * D),
    }


if __name__ == "__main__":
    cases = make_cases()
    fn, _ = cases[os.environ.get("GEMM_CASE", "gate")]
    for _ in range(int(os.environ.get("GEMM_REPS", "6"))):
        fn()
    torch.cuda.synchronize()
    print("done")
