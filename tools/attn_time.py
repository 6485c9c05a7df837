"""ViT-B/16 bs=256 attention forward / backward alone (persistent kernels, dropout 0.1), min of 3
x 20 launches timed by HIP events; ATT_TAG prefixes the line (A/B runs under FERVIT_LIB)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fer-vit_amd"))
import torch  # noqa: E402

from fervit import ops  # noqa: E402


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


B, N, H, dh = 256, 197, 12, 64
g = torch.Generator(device="cuda").manual_seed(0)
qkv = torch.randn(B * N, 3 * H * dh, device="cuda", generator=g).to(torch.bfloat16)
o = torch.empty(B * N, H * dh, device="cuda", dtype=torch.bfloat16)
do = torch.randn(B * N, H * dh, device="cuda", generator=g).to(torch.bfloat16)
dq = torch.empty_like(qkv)
cs = torch.zeros(3 * H * dh, device="cuda")
sv = ops.attention_saved(qkv, B, N, H, dh, dropout=0.1)
fwd = lambda: ops.attention_fwd(qkv, o, sv, B, N, H, dh, dropout=0.1, seed=5)  # noqa: E731
bwd = lambda: ops.attention_bwd(qkv, o, do, sv, dq, B, N, H, dh, dropout=0.1, seed=5, colsum=cs)  # noqa: E731
tf = min(timeit(fwd) for _ in range(3))
fwd()
tb = min(timeit(bwd) for _ in range(3))
print(f"[{os.environ.get('ATT_TAG', '')}] attn fwd {tf:.1f} us  bwd {tb:.1f} us  out_sum {o.float().abs().sum().item():.6e}",
      flush=True)
