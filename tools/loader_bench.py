"""Throughput of the packed-shard loader into HBM (samples/s), with on-device LatentAugment,
vs the reference's per-sample `torch.load` dataset path (LatentFERDataset, one file per
sample, `data/latent_dataset.py:93-116`) measured on a small file sample. Synthetic w+ data."""
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fer-vit_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from fervit.data import PackedLatentDataset, PackedLatentLoader, write_shard  # noqa: E402


def main():
    n = int(os.environ.get("LB_N", 16384))
    d = tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp"))
    rng = np.random.default_rng(0)
    path = os.path.join(d, "train.fwps")
    write_shard(path, rng.standard_normal((n, 18, 512), dtype=np.float32), rng.integers(0, 7, n))
    ds = PackedLatentDataset(path)
    for aug in (None, dict(noise_std=0.1, scale_range=(0.9, 1.1), mask_prob=0.1)):
        ld = PackedLatentLoader(ds, batch_size=256, shuffle=True, seed=1, device="cuda", threads=16, augment=aug)
        for _ in ld:  # warm the page cache / pinned buffers
            pass
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        cnt = 0
        for x, _ in ld:
            cnt += x.shape[0]
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"packed loader (augment={'on' if aug else 'off'}): {cnt / dt:,.0f} samples/s "
              f"({cnt * 18 * 512 * 4 / dt / 1e9:.2f} GB/s into HBM)", flush=True)
    # reference-style: one torch.load per sample file
    fd = os.path.join(d, "pt")
    os.makedirs(fd)
    for i in range(512):
        torch.save({"latent": torch.randn(18, 512), "label": i % 7, "img_path": ""}, os.path.join(fd, f"{i:05d}.pt"))
    files = sorted(os.listdir(fd))
    t0 = time.perf_counter()
    for f in files:
        torch.load(os.path.join(fd, f), map_location="cpu", weights_only=True)
    dt = time.perf_counter() - t0
    print(f"per-sample torch.load (reference dataset path, 1 process): {len(files) / dt:,.0f} samples/s", flush=True)


if __name__ == "__main__":
    main()
