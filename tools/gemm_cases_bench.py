"""Time every ViT-B GEMM case of tools/gemm_case.py (interleaved rounds in one process, min over
rounds). FERVIT_GEMM_DBG=4 in the environment times the main loop alone (no epilogue)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

from gemm_bench import PEAK, timeit  # noqa: E402
from gemm_case import make_cases  # noqa: E402

cases = make_cases()
only = os.environ.get("GB_ONLY")
if only:
    cases = {k: v for k, v in cases.items() if k in only.split(",")}
res = {k: [] for k in cases}
for _ in range(int(os.environ.get("GB_ROUNDS", "3"))):
    for k, (fn, fl) in cases.items():
        res[k].append(timeit(fn))
tag = os.environ.get("GB_TAG", "dbg" + os.environ.get("FERVIT_GEMM_DBG", "0"))
for k, (fn, fl) in cases.items():
    t = min(res[k])
    print(f"[{tag}] {k:12s} {t * 1e3:8.1f} us  {fl / t / 1e9:7.1f} TF ({fl / t / 1e9 / PEAK * 100:4.1f}%)", flush=True)
torch.cuda.synchronize()
