"""Transposed bf16 weight shadow refresh at ViT-B size (every 2-D parameter, one launch)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fer-vit_amd"))
import torch  # noqa: E402

from gemm_bench import timeit  # noqa: E402
from models_fer_vit.image_vit import ImageViT  # noqa: E402

m = ImageViT(img_size=224, embed_dim=768, depth=12, heads=12, mlp_dim=3072).cuda()
flat = m.fer_flat()
flat.half_t_view(m.head.weight)
t = min(timeit(flat.refresh_half_t) for _ in range(3))
n = sum(p.numel() for p in flat.params if p.dim() == 2)
print(f"transpose refresh {t * 1e3:.1f} us for {n / 1e6:.1f} M bf16 ({4 * n / t / 1e6:.0f} GB/s)")
