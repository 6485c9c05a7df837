"""HBM-traffic probe for bench.py's roofline kernel, run UNDER `rocprofv3 --pmc <counter>`.

Runs the bench workload itself -- ViT-B/16 at bs=256, dropout 0.1, label-smoothed CE, fused
AdamW (bench.py `build("vit_base_224")`) -- for `--steps` eager train steps after one warm-up
step; bench.py averages the counter over every gemm_8ph_kernel dispatch in the CSV (the forward
and input-gradient GEMMs of those steps).

usage (bench.py does this before it touches the GPU itself):
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d DIR -o f -- python3 tools/traffic_probe.py
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fer-vit_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2)
    a = ap.parse_args()
    import torch

    import bench

    dev = torch.device("cuda", 0)
    torch.manual_seed(42)
    model, opt, crit, B, shape, _ = bench.build("vit_base_224", dev)
    g = torch.Generator(device=dev).manual_seed(42)
    x = torch.randn(B, *shape, device=dev, generator=g)
    y = torch.randint(0, 7, (B,), device=dev, generator=g)
    for _ in range(1 + a.steps):
        opt.zero_grad()
        crit(model(x), y).backward()
        opt.step()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
