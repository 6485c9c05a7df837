"""GEMM configurations on the small-token shapes (bs=256 x 19 tokens = 4864 rows): LatentViT (E 512,
F 2048) or, with GS_HYBRID=1, the hybrid's timm-B/16 trunk (E 768, F 3072): forward, dgrad
(transposed weights), wgrad; GS_CFGS="auto 3 8 11" forces each tile configuration in turn
(fer_gemm_set_config), interleaved per shape."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fer-vit_amd"))
import torch  # noqa: E402

from fervit import ops  # noqa: E402
from gemm_bench import timeit  # noqa: E402


def main():
    M, E, F = (256 * 19, 768, 3072) if os.environ.get("GS_HYBRID") == "1" else (256 * 19, 512, 2048)
    cfgs = os.environ.get("GS_CFGS")
    if cfgs:  # forward / dgrad shapes under each configuration, interleaved
        from fervit._lib import lib

        g = torch.Generator(device="cuda").manual_seed(0)
        r = lambda *s: torch.randn(*s, device="cuda", generator=g).to(torch.bfloat16)
        x, h = r(M, E), r(M, F)
        cases = {"qkv fwd": (x, r(3 * E, E)), "proj fwd": (x, r(E, E)), "fc1 fwd": (x, r(F, E)), "fc2 fwd": (h, r(E, F)),
                 "fc1 dgrad": (h, r(E, F)), "qkv dgrad": (r(M, 3 * E), r(E, 3 * E))}
        res = {}
        for _ in range(2):
            for k, (a, w) in cases.items():
                for c in cfgs.split():
                    lib().fer_gemm_set_config(-1 if c == "auto" else int(c))
                    t = min(timeit(lambda: ops.linear_fwd(a, w)) for _ in range(3))
                    res[(k, c)] = min(res.get((k, c), 1e9), t)
        lib().fer_gemm_set_config(-1)
        for k, (a, w) in cases.items():
            fl = 2 * a.shape[0] * a.shape[1] * w.shape[0]
            print(f"{k:10s} " + "  ".join(f"cfg {c}: {res[(k, c)] * 1e3:6.1f} us ({fl / res[(k, c)] / 1e9:5.0f} TF)"
                                          for c in cfgs.split()), flush=True)
        return
    g = torch.Generator(device="cuda").manual_seed(0)
    r = lambda *s: torch.randn(*s, device="cuda", generator=g).to(torch.bfloat16)
    x, h = r(M, E), r(M, F)
    shapes = {"qkv fwd": (x, r(3 * E, E)), "out fwd": (x, r(E, E)), "fc1 fwd": (x, r(F, E)), "fc2 fwd": (h, r(E, F))}
    b = {k: torch.zeros(w.shape[0], device="cuda") for k, (a, w) in shapes.items()}
    tag = os.environ.get("FERVIT_GEMM_CFG", "auto")
    tot = 0.0
    for k, (a, w) in shapes.items():
        t = min(timeit(lambda: ops.linear_fwd(a, w, b[k], act="relu")) for _ in range(3))
        tot += t
        fl = 2 * a.shape[0] * a.shape[1] * w.shape[0]
        print(f"[cfg {tag}] {k:8s} {t * 1e3:7.1f} us {fl / t / 1e9:6.1f} TF", flush=True)
    print(f"[cfg {tag}] sum fwd {tot * 1e3:.1f} us", flush=True)
    dys = {"fc1": (h, x), "fc2": (x, h), "qkv": (r(M, 3 * E), x), "out": (x, x)}
    for k, (dy, a) in dys.items():
        gw = torch.empty(dy.shape[1], a.shape[1], device="cuda")
        for split in (True, False):
            t = min(timeit(lambda: ops.linear_wgrad(dy, a, gw, split_ws=split)) for _ in range(3))
            print(f"[cfg {tag}] {k} wgrad split={int(split)} {t * 1e3:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
