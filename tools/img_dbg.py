"""Dump fer_image_augment outputs for the committed fixture (debug aid): gpurun_out/img_dbg.npz."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "fer-vit_amd")]
from fervit.vision import GPUImageTransform  # noqa: E402

g = np.load(os.path.join(ROOT, "tests", "golden", "image_aug.npz"))
S, n = int(g["S"]), int(g["n_src"])
srcs = [g[f"src{i}"] for i in range(n)]
P = g["params"]
tr = GPUImageTransform(S, train=True)([srcs[j % n] for j in range(len(P))], params=torch.from_numpy(P).cuda())
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", "img_dbg.npz"), train=tr.cpu().numpy())
print("ok")
