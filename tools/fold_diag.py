"""Diagnostic for the split-K fold (fer_gemm_set_splitk_fold): one weight-gradient launch with the
separate reduction and one with the fold; for the first elements that differ, the split partials
at that element (from the slab) and the values both paths wrote, to see which combination the
fold computed."""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fer-vit_amd"))
import torch  # noqa: E402

from fervit import ops  # noqa: E402
from fervit._lib import lib  # noqa: E402


def main():
    dev = "cuda"
    M, N, K = 50432, 3072, 768  # tokens, out features, in features: dW [N][K]
    g = torch.Generator(device=dev).manual_seed(M + N + K)
    dy = torch.randn(M, N, device=dev, generator=g).to(torch.bfloat16)
    x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
    outs = []
    for fold in (0, 1):
        lib().fer_gemm_set_splitk_fold(fold)
        c = torch.full((N, K), float("nan"), device=dev)
        ops.linear_wgrad(dy, x, c)
        torch.cuda.synchronize()
        outs.append(c)
    lib().fer_gemm_set_splitk_fold(0)
    ws = [b for k, b in ops.WS.buf.items() if k[1] == 1][0]
    S = 6
    slab = ws[: S * N * K].view(S, N, K)
    ssum = slab[0].clone()
    for s in range(1, S):
        ssum += slab[s]
    print("reduction path == sum of slabs in split order:", torch.equal(ssum, outs[0]))
    d = (outs[1] != outs[0]).nonzero()
    print("differing elements:", d.shape[0])
    for r, c in d[:6].tolist():
        p = slab[:, r, c].tolist()
        print(f"({r},{c}) fold {outs[1][r, c].item():.6g} ref {outs[0][r, c].item():.6g} partials "
              f"{[round(v, 4) for v in p]}")
        # candidate: the fold value equals some partial-sum variant at a neighbour element?
        cands = {}
        for dr in (-1, 0, 1):
            for dc in (-3, -2, -1, 0, 1, 2, 3):
                rr, cc = r + dr, c + dc
                if 0 <= rr < N and 0 <= cc < K:
                    cands[(dr, dc)] = ssum[rr, cc].item()
        hit = [k for k, v in cands.items() if v == outs[1][r, c].item()]
        fv = outs[1][r, c]
        where = (ssum == fv).nonzero()[:4].tolist()
        wslab = (slab == fv).nonzero()[:4].tolist()
        print("   fold value found in the reference sums at", where, "in the slab at", wslab)
        # sums with one split taken from a neighbour / missing
        miss = [s for s in range(S) if abs((ssum[r, c] - slab[s, r, c]).item() - outs[1][r, c].item()) < 1e-3]
        print("   equals sum at neighbour offset:", hit, " equals sum without split:", miss)


if __name__ == "__main__":
    main()
