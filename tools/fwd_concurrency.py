"""What two concurrent half-batch streams buy the ViT-B/16 train forward (and fwd + bwd): is there idle
chip time (GEMM last-round tails, kernel boundaries, VALU-bound attention beside MFMA-bound GEMMs)
that a second stream of independent work fills?

    python tools/fwd_concurrency.py [--reps 10]

Times, on one model (bench.py vit_base_224 build, train mode, dropout 0.1):
  full     forward of the whole batch of 256 on one stream
  seq      forward of two halves (128 + 128) one after the other on one stream
  par      the two halves concurrently, each on its own stream
and the same three for forward + backward (no optimizer step). par < seq by X means X of idle chip time
per step that micro-batch interleaving could recover."""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fer-vit_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    import bench

    dev = torch.device("cuda", 0)
    torch.manual_seed(42)
    model, opt, crit, B, shape, desc = bench.build("vit_base_224", dev)
    g = torch.Generator(device=dev).manual_seed(42)
    x = torch.randn(B, *shape, device=dev, generator=g)
    y = torch.randint(0, 7, (B,), device=dev, generator=g)
    xa, xb, ya, yb = x[: B // 2], x[B // 2:], y[: B // 2], y[B // 2:]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def fwd(xx, yy, bwd):
        loss = crit(model(xx), yy)
        if bwd:
            loss.backward()
        return loss

    def run(mode, bwd):
        opt.zero_grad()
        if mode == "full":
            fwd(x, y, bwd)
        elif mode == "seq":
            fwd(xa, ya, bwd)
            fwd(xb, yb, bwd)
        else:
            cur = torch.cuda.current_stream()
            s1.wait_stream(cur)
            s2.wait_stream(cur)
            with torch.cuda.stream(s1):
                fwd(xa, ya, False)
            with torch.cuda.stream(s2):
                fwd(xb, yb, False)
            cur.wait_stream(s1)
            cur.wait_stream(s2)
            if bwd:  # (the backward of both halves from one loss: autograd runs each on its forward's stream)
                pass

    res = {}
    for bwd in (False,):
        for mode in ("full", "seq", "par"):
            for _ in range(2):
                run(mode, bwd)
            torch.cuda.synchronize()
            ts = []
            for _ in range(a.reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                run(mode, bwd)
                torch.cuda.synchronize()
                ts.append((time.perf_counter() - t0) * 1e3)
            res[(mode, bwd)] = ts
            print(f"{'fwd+bwd' if bwd else 'fwd':8s} {mode:5s} median {statistics.median(ts):8.3f} ms  min {min(ts):8.3f}",
                  flush=True)


if __name__ == "__main__":
    main()
