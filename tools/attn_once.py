"""Run the ViT-B/16 bs=256 attention backward (or forward: ATTN_CASE=fwd) a few times (PMC profiling target)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fer-vit_amd"))
import torch  # noqa: E402

from fervit import ops  # noqa: E402

B, N, H, dh, p = 256, 197, 12, 64, float(os.environ.get("ATTN_P", "0.1"))
D = H * dh
g = torch.Generator(device="cuda").manual_seed(0)
qkv = torch.randn(B * N, 3 * D, device="cuda", generator=g).to(torch.bfloat16)
out = torch.empty(B * N, D, device="cuda", dtype=torch.bfloat16)
dout = torch.randn(B * N, D, device="cuda", generator=g).to(torch.bfloat16)
dqkv = torch.empty_like(qkv)
saved = ops.attention_saved(qkv, B, N, H, dh, dropout=p)
cs = torch.zeros(3 * D, device="cuda")
ops.attention_fwd(qkv, out, saved, B, N, H, dh, dropout=p, seed=5)
for _ in range(4):
    if os.environ.get("ATTN_CASE", "bwd") == "fwd":
        ops.attention_fwd(qkv, out, saved, B, N, H, dh, dropout=p, seed=5)
    else:
        ops.attention_bwd(qkv, out, dout, saved, dqkv, B, N, H, dh, dropout=p, seed=5, colsum=cs)
torch.cuda.synchronize()
print("done")
