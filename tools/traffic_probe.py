"""HBM-traffic probe for bench.py's roofline kernel, run UNDER `rocprofv3 --pmc <counter>`.

Launches the bench's dominant kernel -- the FFN up-projection of ViT-B/16 at bs=256,
Y = GELU(X W1^T + b1) with dropout 0.1 and the pre-activation store, exactly the call
`PostNormLayerFn.forward` makes (fervit/layers.py) -- `--reps` times after warm-up, nothing
else in between, so every gemm dispatch in the counter CSV is that launch.

usage (bench.py does this before it touches the GPU itself):
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d DIR -o f -- python3 tools/traffic_probe.py
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fer-vit_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=256 * 197)
    ap.add_argument("--D", type=int, default=768)
    ap.add_argument("--F", type=int, default=3072)
    ap.add_argument("--reps", type=int, default=6)
    a = ap.parse_args()
    import torch

    from fervit import ops

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(a.M, a.D, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(a.F, a.D, device=dev, generator=g) * 0.03).to(torch.bfloat16)
    b = torch.zeros(a.F, device=dev)
    pre = torch.empty(a.M, a.F, device=dev, dtype=torch.bfloat16)
    out = torch.empty(a.M, a.F, device=dev, dtype=torch.bfloat16)
    for i in range(a.reps):
        ops.linear_fwd(x, w, b, out=out, pre=pre, act="gelu", dropout=0.1, seed=1234 + i, drop_ld=a.F)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
