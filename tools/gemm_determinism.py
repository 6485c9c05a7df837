"""Run-to-run bit equality of the 8-phase GEMM: the same launch repeated must give identical bits.
Residual kind (bias + residual, no dropout), several shapes; prints, per
shape and tile height, how many elements differ between repeats and between the two tile heights,
and where (row % tile height, column % 256) the differences sit."""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fer-vit_amd"))
import torch  # noqa: E402

from fervit import ops  # noqa: E402
from fervit._lib import lib  # noqa: E402


def stress(reps):
    """GD_STRESS=<reps>: the residual launch of the row-tile test's failing case (M 20000, N 768, K 3072,
    automatic configuration: 128^2 tiles) repeated, every repeat compared bit for bit with the first."""
    dev = "cuda"
    M, N, K = 20000, 768, 3072
    g = torch.Generator(device=dev).manual_seed(M + N + K)
    x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev, generator=g) / math.sqrt(K)).to(torch.bfloat16)
    b = torch.randn(N, device=dev, generator=g)
    res = torch.randn(M, N, device=dev, generator=g).to(torch.bfloat16)
    first, nbad = None, 0
    for r in range(reps):
        y = torch.full((M, N), float("nan"), device=dev, dtype=torch.bfloat16)
        ops.linear_fwd(x, w, b, out=y, res=res, dropout=0.0, seed=1234, drop_ld=N)
        torch.cuda.synchronize()
        yi = y.view(torch.int16).clone()
        if first is None:
            first = yi
            continue
        d = yi != first
        if d.any():
            nbad += 1
            idx = d.nonzero()
            bad = y[d].float()
            rows = torch.unique(idx[:, 0])
            cols = torch.unique(idx[:, 1])
            print(f"repeat {r}: {int(d.sum())} elements differ, NaN (unwritten) {int(torch.isnan(bad).sum())}, "
                  f"rows {rows[:16].tolist()} ({len(rows)}), cols {cols.min().item()}..{cols.max().item()} ({len(cols)}), "
                  f"tiles(128) {torch.unique((idx[:, 0] // 128) * 100 + idx[:, 1] // 128)[:8].tolist()}, "
                  f"row%128 {torch.unique(idx[:, 0] % 128)[:16].tolist()}", flush=True)
            good = first.view(torch.bfloat16)[d].float()
            print(f"   got {bad[:6].tolist()} expected {good[:6].tolist()}", flush=True)
    print(f"stress: {nbad} of {reps - 1} repeats differ from the first", flush=True)


def main():
    if os.environ.get("GD_STRESS"):
        stress(int(os.environ["GD_STRESS"]))
        return
    dev = "cuda"
    for (M, N, K) in [(20000, 768, 3072), (50432, 768, 768), (50432, 768, 3072), (20000, 768, 1536)]:
        g = torch.Generator(device=dev).manual_seed(M + N + K)
        x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev, generator=g) / math.sqrt(K)).to(torch.bfloat16)
        b = torch.randn(N, device=dev, generator=g)
        res = torch.randn(M, N, device=dev, generator=g).to(torch.bfloat16)
        reps = []
        for _ in range(3):
            y = torch.full((M, N), float("nan"), device=dev, dtype=torch.bfloat16)
            ops.linear_fwd(x, w, b, out=y, res=res)
            torch.cuda.synchronize()
            reps.append(y.view(torch.int16).clone())
        d = [(reps[0] != r).sum().item() for r in reps[1:]]
        print(f"M {M} N {N} K {K}: repeats differing elements {d}", flush=True)
if __name__ == "__main__":
    main()
