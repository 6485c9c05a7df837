"""Phase timeline of the 8-phase GEMM from the diagnostic stamp build (FER_GEMM_STAMPS):
  FERVIT_LIB=fer-vit_amd/fervit/libfervit_st.so python tools/gemm_stamps.py [case]
Prints, for wave 0 (group A) and wave 4 (group B) of workgroup 0's second tile, the cycles of
each phase's load segment, barrier-1 wait, MFMA segment and barrier-2 wait (s_memtime), and the
prologue / epilogue spans. Shares only: the stamps' lgkmcnt(0) drains change the schedule."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fer-vit_amd"))
import torch  # noqa: E402

from fervit import ops  # noqa: E402
from fervit._lib import lib  # noqa: E402


def main():
    case = sys.argv[1] if len(sys.argv) > 1 else "fc1"
    dev = "cuda"
    M, D, F = 256 * 197, 768, 3072
    g = torch.Generator(device=dev).manual_seed(0)
    r = lambda *s: torch.randn(*s, device=dev, generator=g, dtype=torch.bfloat16)
    x, w1, w2 = r(M, D), r(F, D) * 0.03, r(D, F) * 0.03
    h = r(M, F)
    b1 = torch.zeros(F, device=dev)
    pre = torch.empty(M, F, device=dev, dtype=torch.bfloat16)
    if case == "fc1":
        fn = lambda: ops.linear_fwd(x, w1)
    elif case == "fc1fused":
        fn = lambda: ops.linear_fwd(x, w1, b1, pre=pre, act="gelu", dropout=0.1, seed=7)
    elif case == "fc1gate":
        fn = lambda: ops.linear_fwd(x, w1, b1, pre=pre, pre_gate=True, act="gelu", dropout=0.1, seed=7)
    elif case == "fc2res":  # fc2 fwd with bias + dropout + residual (K = 3072)
        fn = lambda: ops.linear_fwd(h, w2, b1[:D], res=x, dropout=0.1, seed=7)
    else:  # fc2: K = 3072
        fn = lambda: ops.linear_fwd(h, w2)
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    L = lib()
    n = 2 * (4 + 256)
    buf = (ctypes.c_ulonglong * n)()
    L.fer_debug_gemm_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    assert L.fer_debug_gemm_stamps(ctypes.addressof(buf), n) == 0
    ep = (ctypes.c_ulonglong * 32)()
    L.fer_debug_gemm_ep_stamps.argtypes = [ctypes.c_void_p]
    assert L.fer_debug_gemm_ep_stamps(ctypes.addressof(ep)) == 0
    names = ["stage0", "finish0", "stage1", "finish1", "stage2", "finish2", "stage3", "finish3"]
    for w in range(2):
        e = ep[w * 16:(w + 1) * 16]
        print(f"epilogue wave {4 * w} (last tile of WG 0): total {e[8] - e[0]} cyc: " +
              "  ".join(f"{nm} {e[i + 1] - e[i]}" for i, nm in enumerate(names)))
    for w in range(2):
        s = buf[w * 260:(w + 1) * 260]
        t0 = s[0]
        print(f"wave {4 * w}: prologue {s[1] - s[0]} cyc, main loop {s[2] - s[1]}, epilogue {s[3] - s[2]}")
        nk = 16 if case.startswith("fc2") else 12
        tot = [0, 0, 0, 0]
        cnt = 0
        for T in range(nk):
            row = []
            for q in range(4):
                i = 4 + (T * 4 + q) * 4
                a, b_, c, d = s[i:i + 4]
                nxt = s[i + 4] if (T * 4 + q + 1) < 64 and s[i + 4] else None
                if not a or not b_ or not c or not d:
                    continue
                seg = [b_ - a, c - b_, d - c, (nxt - d) if nxt else 0]
                row.append("/".join(str(v) for v in seg))
                if 0 < T < nk - 1 and nxt:
                    tot = [u + v for u, v in zip(tot, seg)]
                    cnt += 1
            print(f"  T={T:2d} load/bar1/mfma/bar2: " + "  ".join(row))
        if cnt:
            avg = [v / cnt for v in tot]
            ph = sum(avg)
            print(f"  steady-state avg per phase: load {avg[0]:.0f}  bar1 {avg[1]:.0f}  mfma {avg[2]:.0f}  "
                  f"bar2 {avg[3]:.0f}  = {ph:.0f} cyc (MFMA segment share {avg[2] / ph:.2f})")


if __name__ == "__main__":
    main()
