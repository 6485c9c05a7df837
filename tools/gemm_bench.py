"""GEMM microbenchmark on the ViT-B/16 bs=256 shapes: libfervit bf16 GEMM (plain and
with the real epilogues) vs torch.matmul (hipBLASLt) as a known-good reference.
Interleaved rounds in one process (cdna guide §5.4 rule 24); random N(0,1) data."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fer-vit_amd"))
import torch  # noqa: E402

from fervit import ops  # noqa: E402

PEAK = 2516.6


def timeit(fn, reps=20):
    s = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    a.record(s)
    for _ in range(reps):
        fn()
    b.record(s)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    dev = "cuda"
    M, D, F = 256 * 197, 768, 3072
    g = torch.Generator(device=dev).manual_seed(0)
    r = lambda *s: torch.randn(*s, device=dev, generator=g, dtype=torch.bfloat16)
    x, w1, w2, wqkv = r(M, D), r(F, D) * 0.03, r(D, F) * 0.03, r(3 * D, D) * 0.03
    h, dF = r(M, F), r(M, F)
    b1 = torch.zeros(F, device=dev)
    pre = torch.empty(M, F, device=dev, dtype=torch.bfloat16)
    gw = torch.empty(F, D, device=dev)
    w2t, w1t = w2.t().contiguous(), w1.t().contiguous()  # [F, D], [D, F]
    wo, bo = r(D, D) * 0.03, torch.zeros(D, device=dev)
    q3, wqkvt = r(M, 3 * D), wqkv.t().contiguous()  # dqkv [M, 3D], W_qkv^T [D, 3D]
    gwq, gwo, gw2 = torch.empty(3 * D, D, device=dev), torch.empty(D, D, device=dev), torch.empty(D, F, device=dev)
    out_f = torch.empty(M, F, device=dev, dtype=torch.bfloat16)
    out_d = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    cs = torch.zeros(F, device=dev)
    fused = dict(aux=pre, aux_act="gelu", dropout=0.1, seed=9, drop_ld=F, colsum=cs)
    cases = {
        "fc1 fwd plain": (lambda: ops.linear_fwd(x, w1), 2 * M * F * D, lambda: x @ w1.t()),
        "fc1 fwd +bias+gelu+drop+pre": (lambda: ops.linear_fwd(x, w1, b1, pre=pre, act="gelu", dropout=0.1, seed=7),
                                         2 * M * F * D, None),
        "fc1 fwd +bias+gelu+drop+gate": (lambda: ops.linear_fwd(x, w1, b1, pre=pre, pre_gate=True, act="gelu",
                                                                 dropout=0.1, seed=7), 2 * M * F * D, None),
        "fc1 fwd +bias": (lambda: ops.linear_fwd(x, w1, b1, out=out_f), 2 * M * F * D, None),
        "fc1 fwd +bias+gelu": (lambda: ops.linear_fwd(x, w1, b1, out=out_f, act="gelu"), 2 * M * F * D, None),
        "fc1 fwd +bias+relu+pre": (lambda: ops.linear_fwd(x, w1, b1, out=out_f, act="relu", pre=pre), 2 * M * F * D, None),
        "fc1 fwd +bias+gelu+drop": (lambda: ops.linear_fwd(x, w1, b1, out=out_f, act="gelu", dropout=0.1, seed=7),
                                    2 * M * F * D, None),
        "fc2 fwd plain (K=3072)": (lambda: ops.linear_fwd(h, w2), 2 * M * F * D, lambda: h @ w2.t()),
        "qkv fwd plain": (lambda: ops.linear_fwd(x, wqkv), 2 * M * 3 * D * D, lambda: x @ wqkv.t()),
        "fc2 dgrad (B MN)": (lambda: ops.linear_dgrad(x, w2), 2 * M * F * D, lambda: x @ w2),
        "fc2 dgrad (B KC, W^T copy)": (lambda: ops.linear_fwd(x, w2t, out=out_f), 2 * M * F * D, None),
        "fc2 dgrad fused (B MN)": (lambda: ops.linear_dgrad(x, w2, out=out_f, **fused), 2 * M * F * D, None),
        "fc2 dgrad fused (B KC)": (lambda: ops.linear_fwd(x, w2t, out=out_f, **fused), 2 * M * F * D, None),
        "fc2 dgrad gate-mul (B KC)": (lambda: ops.linear_fwd(x, w2t, out=out_f, aux=pre, aux_act="mul", colsum=cs),
                                      2 * M * F * D, None),
        "fc1 dgrad +res (B MN, K=3072)": (lambda: ops.linear_dgrad(h, w1, out=out_d, res=x), 2 * M * F * D, None),
        "fc1 dgrad +res (B KC, K=3072)": (lambda: ops.linear_fwd(h, w1t, out=out_d, res=x), 2 * M * F * D, None),
        "fc1 wgrad (MN,MN splitK)": (lambda: ops.linear_wgrad(dF, x, gw), 2 * M * F * D, lambda: dF.t() @ x),
        "qkv wgrad (MN,MN splitK)": (lambda: ops.linear_wgrad(q3, x, gwq), 2 * M * 3 * D * D, None),
        "out wgrad (MN,MN splitK)": (lambda: ops.linear_wgrad(x, x, gwo), 2 * M * D * D, None),
        "fc2 wgrad (MN,MN splitK)": (lambda: ops.linear_wgrad(x, dF, gw2), 2 * M * F * D, None),
        "out-proj fwd +bias+drop+res": (lambda: ops.linear_fwd(x, wo, bo, out=out_d, res=x, dropout=0.1, seed=3),
                                        2 * M * D * D, None),
        "fc2 fwd +bias+drop+res (K=3072)": (lambda: ops.linear_fwd(h, w2, bo, out=out_d, res=x, dropout=0.1, seed=3),
                                            2 * M * F * D, None),
        "qkv dgrad +res (B KC, K=2304)": (lambda: ops.linear_fwd(q3, wqkvt, out=out_d, res=x), 2 * M * 3 * D * D, None),
    }
    cfg = os.environ.get("GB_CFG")  # force one tile configuration (fer_gemm_set_config)
    if cfg is not None:
        from fervit._lib import lib

        lib().fer_gemm_set_config(int(cfg))
    only = os.environ.get("GB_ONLY")
    if only:
        cases = {k: v for k, v in cases.items() if only in k}
    rows = [(None, None)]

    res = {(k, rt): [] for k in cases for rt, _ in rows}
    ref = {k: [] for k in cases}
    for _ in range(3):
        for k, (fn, fl, tf) in cases.items():
            for rt, setv in rows:
                if setv is not None:
                    setv()
                res[(k, rt)].append(timeit(fn))
            if tf is not None:
                ref[k].append(timeit(tf))
    tag = cfg if cfg is not None else "auto"
    for k, (fn, fl, tf) in cases.items():
        for rt, _ in rows:
            t = min(res[(k, rt)])
            rtag = f" {rt}" if rt is not None else ""
            line = (f"[cfg {tag}{rtag}] {k:32s} ours {t * 1e3:8.1f} us  {fl / t / 1e9:7.1f} TF "
                    f"({fl / t / 1e9 / PEAK * 100:4.1f}%)")
            if ref[k] and rt == rows[0][0]:
                tr = min(ref[k])
                line += f"   hipBLASLt {tr * 1e3:8.1f} us {fl / tr / 1e9:7.1f} TF"
            print(line, flush=True)


if __name__ == "__main__":
    main()
