"""Debug: compare the stored attention dropout keep bits with the host hash (one small case)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fer-vit_amd")); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np, torch
from fervit import ops
from dropmask import keep_mask
B, N, H, dh, p, seed = 1, 10, 1, 48, 0.5, 4242
qkv = torch.randn(B * N, 3 * H * dh, device="cuda").to(torch.bfloat16)
out = torch.empty(B * N, H * dh, device="cuda", dtype=torch.bfloat16)
saved = ops.attention_saved(qkv, B, N, H, dh, dropout=p)
ops.attention_fwd(qkv, out, saved, B, N, H, dh, dropout=p, seed=seed)
off = (B * H * N + 63) // 64 * 64
w = saved[off:off + 32].view(torch.int32).cpu().numpy().view(np.uint32)
keep = keep_mask(seed, (B, H, N, N + (N & 1)), p)[..., :N].reshape(N, N)  # [q][k]
for j in range(N):
    want = sum(int(keep[q, j]) << q for q in range(N))
    print(j, f"{int(w[j]) & ((1 << N) - 1):010b}"[::-1], f"{want:010b}"[::-1])
