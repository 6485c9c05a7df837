"""Every GEMM of one latent_vit encoder layer (cfg 2: bs 256 x 19 tokens = 4864 rows, D 512, F 2048,
ReLU FFN, dropout 0.1) alone on the chip, with the epilogue the layer uses: forward, input gradient
(dgrad through the transposed bf16 weight) and weight gradient (MN x MN, fp32 out, split-K).
GB_ONLY=a,b selects cases; GB_TAG prefixes the lines (A/B runs under FERVIT_GEMM_CFG etc.)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fer-vit_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

from fervit import ops  # noqa: E402
from gemm_bench import timeit  # noqa: E402


def main():
    M, D, F = 256 * 19, 512, 2048
    g = torch.Generator(device="cuda").manual_seed(0)
    r = lambda *s: torch.randn(*s, device="cuda", generator=g).to(torch.bfloat16)
    x, h = r(M, D), r(M, F)
    wqkv, wo, w1, w2 = r(3 * D, D), r(D, D), r(F, D), r(D, F)
    w1t, w2t, wqkvt = r(D, F), r(F, D), r(D, 3 * D)
    bq, bo, b1, b2 = (torch.zeros(n, device="cuda") for n in (3 * D, D, F, D))
    gate = torch.empty(M, F, device="cuda", dtype=torch.bfloat16)
    cs = torch.zeros(F, device="cuda")
    dq = r(M, 3 * D)
    gw = {n: torch.zeros(*s, device="cuda") for n, s in (("qkv", (3 * D, D)), ("o", (D, D)), ("1", (F, D)),
                                                         ("2", (D, F)))}
    hT, xT = r(F, M), r(D, M)  # token-contiguous copies: the weight gradient as a K x K GEMM (experiment)
    cases = {
        "qkv_fwd": (lambda: ops.linear_fwd(x, wqkv, bq), 2 * M * 3 * D * D),
        "out_fwd": (lambda: ops.linear_fwd(x, wo, bo, res=x, dropout=0.1, seed=3, drop_ld=D), 2 * M * D * D),
        "fc1_fwd": (lambda: ops.linear_fwd(x, w1, b1, pre=gate, pre_gate=True, act="relu", dropout=0.1, seed=5,
                                           drop_ld=F), 2 * M * F * D),
        "fc1_fwd_nodrop": (lambda: ops.linear_fwd(x, w1, b1, pre=gate, pre_gate=True, act="relu"), 2 * M * F * D),
        "fc1_fwd_gelu": (lambda: ops.linear_fwd(x, w1, b1, pre=gate, pre_gate=True, act="gelu", dropout=0.1, seed=5,
                                                drop_ld=F), 2 * M * F * D),
        "fc2_fwd": (lambda: ops.linear_fwd(h, w2, b2, res=x, dropout=0.1, seed=7, drop_ld=D), 2 * M * F * D),
        "fc2_dgrad": (lambda: ops.linear_fwd(x, w2t, aux=gate, aux_act="mul", colsum=cs), 2 * M * F * D),
        "fc1_dgrad": (lambda: ops.linear_fwd(h, w1t, res=x), 2 * M * F * D),
        "out_dgrad": (lambda: ops.linear_fwd(x, wo), 2 * M * D * D),
        "qkv_dgrad": (lambda: ops.linear_fwd(dq, wqkvt, res=x), 2 * M * 3 * D * D),
        "qkv_wgrad": (lambda: ops.linear_wgrad(dq, x, gw["qkv"]), 2 * M * 3 * D * D),
        "out_wgrad": (lambda: ops.linear_wgrad(x, x, gw["o"]), 2 * M * D * D),
        "fc1_wgrad": (lambda: ops.linear_wgrad(h, x, gw["1"]), 2 * M * F * D),
        "fc2_wgrad": (lambda: ops.linear_wgrad(x, h, gw["2"]), 2 * M * F * D),
        "fc1_wgrad_kk": (lambda: ops.gemm(hT, xT, gw["1"], M=F, N=D, K=M), 2 * M * F * D),
        # the layer's four weight gradients as one grouped launch (what the latent layers run)
        "wgrad_group": (lambda: ops.linear_wgrad_group([(dq, x, gw["qkv"], False), (x, x, gw["o"], False),
                                                        (h, x, gw["1"], False), (x, h, gw["2"], False)]),
                        2 * M * (3 * D * D + D * D + 2 * F * D)),
    }
    only = os.environ.get("GB_ONLY")
    tag = os.environ.get("GB_TAG", "")
    tot = 0.0
    for k, (fn, fl) in cases.items():
        if only and k not in only.split(","):
            continue
        t = min(timeit(fn) for _ in range(3))
        if not k.endswith(("nodrop", "gelu", "_kk", "_group")):
            tot += t
        print(f"[{tag}] {k:15s} {t * 1e3:7.1f} us {fl / t / 1e12 * 1e3:7.1f} TF", flush=True)
    print(f"[{tag}] layer sum {tot * 1e3:.1f} us", flush=True)


if __name__ == "__main__":
    main()
