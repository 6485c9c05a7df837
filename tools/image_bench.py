"""Throughput of the ImageViT transforms: fer_image_augment on device (sources resident in HBM,
HIP-event timed) and end to end from host arrays (packing + pinned H2D + kernel), against the
reference's per-image Pillow/torchvision pipeline on one host core (oracle/image_oracle.py)."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "fer-vit_amd"), os.path.join(ROOT, "oracle")]
from fervit import ops  # noqa: E402
from fervit._lib import check, lib  # noqa: E402
from fervit.vision import GPUImageTransform  # noqa: E402


def bench(shape, B=256, S=224, iters=20):
    rng = np.random.default_rng(0)
    srcs = [rng.integers(0, 256, shape, dtype=np.uint8) for _ in range(B)]
    res = {"source": "x".join(map(str, shape)), "B": B, "S": S}
    for train in (False, True):
        t = GPUImageTransform(S, train=train)
        t(srcs)  # warm-up, draws params
        src, offs, hwc = t.pack(srcs)
        out = torch.empty(B, 3, S, S, device="cuda")
        prm = t.last_params if train else None
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(iters):
            check(lib().fer_image_augment(src.data_ptr(), offs.data_ptr(), hwc.data_ptr(), B, S,
                                          prm.data_ptr() if prm is not None else None, int(train), t.mean, t.std,
                                          out.data_ptr(), ops.stream()), "image_augment")
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / iters
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            t(srcs)
        torch.cuda.synchronize()
        e2e = (time.perf_counter() - t0) / 5
        k = "train" if train else "val"
        res[k + "_kernel_ms"] = round(ms, 3)
        res[k + "_kernel_img_s"] = round(B / ms * 1e3)
        res[k + "_e2e_img_s"] = round(B / e2e)
        res[k + "_out_GBps"] = round(B * 3 * S * S * 4 / ms / 1e6, 1)
    import image_oracle as O
    from PIL import Image

    ims = [Image.fromarray(a if a.shape[2] == 3 else a[:, :, 0]) for a in srcs[:64]]
    P = O.random_params(64, S, rng)
    t0 = time.perf_counter()
    for im, p in zip(ims, P):
        O.normalize(O.train_uint8(im, S, p))
    res["pillow_train_img_s_1core"] = round(64 / (time.perf_counter() - t0))
    t0 = time.perf_counter()
    for im in ims:
        O.normalize(O.val_uint8(im, S))
    res["pillow_val_img_s_1core"] = round(64 / (time.perf_counter() - t0))
    return res


if __name__ == "__main__":
    for shape in ((48, 48, 1), (256, 256, 3)):
        print(json.dumps(bench(shape)), flush=True)
