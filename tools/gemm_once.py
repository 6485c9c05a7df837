"""Run one ViT-B GEMM a few times (PMC profiling target): GEMM_CASE=fc1 (K 768, plain) | fc2 (K 3072, plain) |
fc1_fused (bias + GELU + dropout + pre) |
fc1_gate (the model's fc1 forward: bias + GELU + dropout + gate, pre_gate). GEMM_CFG=<n>: force library config n (fer_gemm_set_config)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fer-vit_amd"))
import torch  # noqa: E402

from fervit import ops  # noqa: E402
from fervit._lib import lib  # noqa: E402

if os.environ.get("GEMM_CFG"):
    lib().fer_gemm_set_config(int(os.environ["GEMM_CFG"]))

M, D, F = 256 * 197, 768, 3072
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.randn(M, D, device="cuda", generator=g).to(torch.bfloat16)
w = (torch.randn(F, D, device="cuda", generator=g) * 0.03).to(torch.bfloat16)
b = torch.zeros(F, device="cuda")
pre = torch.empty(M, F, device="cuda", dtype=torch.bfloat16)
out = torch.empty(M, F, device="cuda", dtype=torch.bfloat16)
case = os.environ.get("GEMM_CASE", "fc1")
if case == "fc2":
    h = torch.randn(M, F, device="cuda", generator=g).to(torch.bfloat16)
    w2 = (torch.randn(D, F, device="cuda", generator=g) * 0.03).to(torch.bfloat16)
    y2 = torch.empty(M, D, device="cuda", dtype=torch.bfloat16)
for _ in range(6):
    if case == "fc1":
        ops.linear_fwd(x, w, out=out)
    elif case == "fc2":
        ops.linear_fwd(h, w2, out=y2)
    elif case == "fc1_gate":
        ops.linear_fwd(x, w, b, out=out, pre=pre, pre_gate=True, act="gelu", dropout=0.1, seed=7)
    else:
        ops.linear_fwd(x, w, b, out=out, pre=pre, act="gelu", dropout=0.1, seed=7)
torch.cuda.synchronize()
print("done")
