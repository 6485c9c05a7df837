"""GEMM / attention time while a few CUs are held by another stream's workgroups (the way RCCL's
all-reduce kernels hold CUs during the DDP-overlapped backward). tools/micro/libhog.so spins
NB workgroups of 64 KB LDS on a side stream; the measured kernel starts right after them.
  python tools/hog_bench.py [nb ...]      (FERVIT_GEMM_NOPERSIST=1 for the non-persistent GEMM)"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fer-vit_amd"))
import torch  # noqa: E402

from fervit import ops  # noqa: E402


def main():
    hog = ctypes.CDLL(os.path.join(ROOT, "tools", "micro", "libhog.so"))
    hog.hog_launch.argtypes = [ctypes.c_int, ctypes.c_longlong, ctypes.c_void_p, ctypes.c_void_p]
    dev = "cuda"
    M, D, F = 256 * 197, 768, 3072
    g = torch.Generator(device=dev).manual_seed(0)
    r = lambda *s: torch.randn(*s, device=dev, generator=g, dtype=torch.bfloat16)
    x, w1, w2, h = r(M, D), r(F, D) * 0.03, r(D, F) * 0.03, r(M, F)
    res = r(M, D)
    b1, b2 = torch.zeros(F, device=dev), torch.zeros(D, device=dev)
    pre = torch.empty(M, F, device=dev, dtype=torch.bfloat16)
    B, N, H, dh = 256, 197, 12, 64
    qkv = r(M, 3 * D)
    ao, dqkv = torch.empty(M, D, device=dev, dtype=torch.bfloat16), torch.empty_like(qkv)
    lse = ops.attention_saved(qkv, B, N, H, dh, dropout=0.1)
    cases = {
        "fc1 fwd gelu": lambda: ops.linear_fwd(x, w1, b1, pre=pre, act="gelu", dropout=0.1, seed=7),
        "fc2 fwd res": lambda: ops.linear_fwd(h, w2, b2, res=res, dropout=0.1, seed=9),
        "fc1 wgrad": lambda: ops.linear_wgrad(h, x, gw),
        "attn fwd": lambda: ops.attention_fwd(qkv, ao, lse, B, N, H, dh, dropout=0.1, seed=5),
        "attn bwd": lambda: ops.attention_bwd(qkv, ao, res, lse, dqkv, B, N, H, dh, dropout=0.1, seed=5),
    }
    gw = torch.empty(F, D, device=dev)
    sink = torch.zeros(1, device=dev, dtype=torch.int32)
    side = torch.cuda.Stream()
    nbs = [int(a) for a in sys.argv[1:]] or [0, 16, 32]
    for name, fn in cases.items():
        fn()
        torch.cuda.synchronize()
        line = []
        for nb in nbs:
            ts = []
            for _ in range(7):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                if nb:
                    hog.hog_launch(nb, 4_000_000, sink.data_ptr(), ctypes.c_void_p(side.cuda_stream))
                torch.cuda._sleep(100_000)  # the hog is resident before the measured kernel starts
                a.record()
                fn()
                b.record()
                torch.cuda.synchronize()
                ts.append(a.elapsed_time(b) * 1e3)
            ts.sort()
            line.append(f"hog {nb:3d}: {ts[len(ts) // 2]:7.1f} us")
        print(f"{name:14s} " + "   ".join(line), flush=True)


if __name__ == "__main__":
    main()
