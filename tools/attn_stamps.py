"""Timeline of the persistent attention forward from the diagnostic stamp build (FER_ATTN_STAMPS):
  FERVIT_LIB=fer-vit_amd/fervit/libfervit_st.so python tools/attn_stamps.py
Workgroup 0, units 2 and 3: per wave, cycles from the unit's start to each stamp (consumers: per key
block, before / after its softmax + P.V; producer: DMA issued, DMA landed; all: before / after the
unit's barrier)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fer-vit_amd"))
import torch  # noqa: E402

from fervit import ops  # noqa: E402
from fervit._lib import lib  # noqa: E402


def main():
    B, N, H, dh = 256, 197, 12, 64
    D = H * dh
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = torch.randn(B * N, 3 * D, device="cuda", generator=g).to(torch.bfloat16)
    out = torch.empty(B * N, D, device="cuda", dtype=torch.bfloat16)
    lib().fer_attention_set_fwd_kernel(1)  # the stamped persistent forward (the automatic choice at p > 0 is the occupancy form)
    for p in (0.1, 0.0):
        lse = ops.attention_saved(qkv, B, N, H, dh, dropout=p)
        for _ in range(3):
            ops.attention_fwd(qkv, out, lse, B, N, H, dh, dropout=p, seed=5)
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * (9 * 64))()
        assert lib().fer_debug_attn_stamps(buf) == 0
        st = [list(buf[w * 64:(w + 1) * 64]) for w in range(9)]
        print(f"p={p}")
        for u in (0, 1):
            base = min(st[w][u * 32] for w in range(8) if st[w][u * 32])
            for w in range(8):
                row = st[w][u * 32:u * 32 + 32]
                if w == 7:
                    pts = [("dma_issued", 1), ("dma_landed", 2), ("bar_out", 21)]
                else:
                    pts = [(f"kb{kb}", 2 + 2 * kb) for kb in range(7)] + [("end", 20), ("bar_out", 21)]
                txt = " ".join(f"{n}={row[i] - base:6d}" for n, i in pts if row[i])
                print(f"  unit{u} w{w} start={row[0] - base:6d} {txt}")
        wg_stats()
    lib().fer_attention_set_fwd_kernel(0)


def wg_stats():
    """Per-workgroup units, core cycles and wall time (s_memrealtime, 100 MHz) of the last forward."""
    buf = (ctypes.c_ulonglong * (1024 * 5))()
    if not hasattr(lib(), "fer_debug_attn_wg_stats") or lib().fer_debug_attn_wg_stats(buf) != 0:
        return
    rows = [buf[i * 5:(i + 1) * 5] for i in range(1024)]
    rows = [r for r in rows if r[0]]
    units = [r[0] for r in rows]
    cyc = [r[2] - r[1] for r in rows]
    wall = [(r[4] - r[3]) / 100.0 for r in rows]  # us
    t0 = min(r[3] for r in rows)
    last = max(r[4] for r in rows)
    print(f"  WGs {len(rows)}  units/WG min {min(units)} max {max(units)}  kernel span {(last - t0) / 100.0:.1f} us  "
          f"WG wall min {min(wall):.1f} max {max(wall):.1f} us  clock {sum(cyc) / sum(wall) / 1e3:.2f} GHz  "
          f"cycles/unit {sum(cyc) / sum(units):.0f}")




def bwd():
    B, N, H, dh = 256, 197, 12, 64
    D = H * dh
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = torch.randn(B * N, 3 * D, device="cuda", generator=g).to(torch.bfloat16)
    out = torch.empty(B * N, D, device="cuda", dtype=torch.bfloat16)
    dout = torch.randn(B * N, D, device="cuda", generator=g).to(torch.bfloat16)
    dqkv = torch.empty(B * N, 3 * D, device="cuda", dtype=torch.bfloat16)
    lse = ops.attention_saved(qkv, B, N, H, dh, dropout=0.1)
    ops.attention_fwd(qkv, out, lse, B, N, H, dh, dropout=0.1, seed=5)
    for _ in range(3):
        ops.attention_bwd(qkv, out, dout, lse, dqkv, B, N, H, dh, dropout=0.1, seed=5)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (8 * 128))()
    assert lib().fer_debug_attn_bwd_stamps(buf) == 0
    st = [list(buf[w * 128:(w + 1) * 128]) for w in range(8)]
    print("bwd p=0.1 (per step: s=start v=P/dS VALU done t=dS written + dV/dK operand reads issued d=dV/dK MFMAs issued "
          "b1=after barrier 1 q=dQ done b2=after barrier 2)")
    for u in (0, 1):
        o = u * 64
        base = min(st[w][o] for w in range(7) if st[w][o])
        for w in range(7):
            row = st[w][o:o + 64]
            parts = []
            for i in range(7):
                s0, d, b1, q, b2, v, t = (row[1 + 7 * i + j] - base for j in range(7))
                parts.append(f"[{s0}|{v}|{t}|{d}|{b1}|{q}|{b2}]")
            print(f"  unit{u} w{w} " + " ".join(parts) + f" last_loads={row[54] - base} epi: waited={row[50] - base} "
                  f"dq={row[51] - base} cs={row[52] - base} stg={row[53] - base} end={row[60] - base} out={row[61] - base}")



if __name__ == "__main__":
    main()
    bwd()
