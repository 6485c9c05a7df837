"""Tensor-level wrappers around the C ABI (one call = one or two kernel launches).

Every wrapper takes device tensors, checks shapes/strides on the host before the
launch (kernels assume what the host verified), and enqueues on PyTorch's current
HIP stream. Nothing here has a CPU path.
"""
from __future__ import annotations

import math
from typing import Optional

import torch

from . import _lib
from ._lib import Epilogue, GemmDesc, check, lib

ACT = {"none": 0, "gelu": 1, "relu": 2, "mul": 3}  # "mul": aux_act only (v *= aux)
PRE_GATE = 16  # act flag: `pre` receives act'(pre) * keep * drop_scale (include/fervit.h)

# Optional callable(desc, epilogue, launch) used by bench.py to bracket launches with HIP events.
LAUNCH_PROBE = None


def dcode(t: torch.Tensor) -> int:
    if t.dtype == torch.bfloat16:
        return 0
    if t.dtype == torch.float32:
        return 1
    raise TypeError(f"fervit: unsupported activation dtype {t.dtype}")


def ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _dev(t: torch.Tensor) -> None:
    if not t.is_cuda:
        raise RuntimeError("fervit: the HIP path needs tensors on a ROCm device (no CPU fallback)")


# ------------------------------------------------------------------ workspace
class _Workspace:
    """Grow-only fp32 scratch per (device, slot, stream): users on one stream are ordered by it,
    and the weight-gradient stream (runtime.WGRAD) gets buffers of its own."""

    def __init__(self):
        self.buf = {}

    def get(self, nbytes: int, device, slot: int = 0) -> torch.Tensor:
        key = (device, slot, torch.cuda.current_stream(device).cuda_stream)
        b = self.buf.get(key)
        n = max(1, (int(nbytes) + 3) // 4)
        if b is None or b.numel() < n:
            b = torch.empty(int(n * 1.25) + 1024, dtype=torch.float32, device=device)
            self.buf[key] = b
        return b


WS = _Workspace()


def drop_args(p: float):
    """(thresh, scale): an element is dropped iff its 16-bit uniform < thresh = round(p*65536)."""
    if p <= 0.0:
        return 0, 1.0
    if p >= 1.0:
        return 65536, 0.0
    thr = max(1, min(65535, int(round(p * 65536.0))))
    return thr, 1.0 / (1.0 - p)


# ------------------------------------------------------------------ GEMM
def gemm(A: torch.Tensor, B: torch.Tensor, out: torch.Tensor, *, a_kc: bool = True, b_kc: bool = True,
         M: int, N: int, K: int, lda: Optional[int] = None, ldb: Optional[int] = None, ldc: Optional[int] = None,
         bias: Optional[torch.Tensor] = None, act: str = "none", pre: Optional[torch.Tensor] = None,
         res: Optional[torch.Tensor] = None, dropout: float = 0.0, seed: int = 0, drop_ld: Optional[int] = None,
         aux: Optional[torch.Tensor] = None, aux_act: str = "none", alpha: float = 1.0, accumulate: bool = False,
         post_scale: Optional[torch.Tensor] = None, split_ws: bool = True,
         colsum: Optional[torch.Tensor] = None, colsum_accumulate: bool = False,
         pre_gate: bool = False) -> torch.Tensor:
    """out[m][n] = epilogue(sum_k A(m,k) B(n,k)); see include/fervit.h for the layouts.
    colsum: optional fp32 [N] receiving (or, with colsum_accumulate, adding) sum_m out[m][n].
    pre_gate: `pre` receives act'(pre) * dropout keep * scale (consumed by aux_act="mul")."""
    _dev(A)
    if A.dtype != B.dtype:
        raise TypeError("gemm: A and B dtypes differ")
    d = GemmDesc()
    d.dtype = dcode(A)
    d.A, d.B = A.data_ptr(), B.data_ptr()
    d.lda = lda if lda is not None else (K if a_kc else M)
    d.ldb = ldb if ldb is not None else (K if b_kc else N)
    d.a_kc, d.b_kc = int(a_kc), int(b_kc)
    d.M, d.N, d.K = M, N, K
    t256 = -(-M // 256) * -(-N // 256)
    if colsum is not None:
        w = WS.get(lib().fer_gemm_colsum_ws(M, N), A.device, slot=1)
        d.ws, d.ws_bytes = w.data_ptr(), w.numel() * 4
    elif split_ws and d.dtype == 0 and K >= 1024 and t256 < 256:
        # split-K slabs: the library targets ~one 256x256 workgroup per CU (or 512 128^2 ones)
        nb = 4 * M * N * min(32, max(2, 512 // t256)) + 4 * (-(-M // 128) * -(-N // 128)) + 256  # + tile tickets
        w = WS.get(nb, A.device, slot=1)
        d.ws, d.ws_bytes = w.data_ptr(), w.numel() * 4
    e = Epilogue()
    e.c = out.data_ptr()
    e.ldc = ldc if ldc is not None else N
    e.c_f32 = int(out.dtype == torch.float32)
    e.accumulate = int(accumulate)
    e.alpha = alpha
    e.bias = ptr(bias)
    e.act = ACT[act] | (PRE_GATE if pre_gate else 0)
    e.pre = ptr(pre)
    e.ldp = N if pre is None else pre.stride(0)
    e.res = ptr(res)
    e.ldr = N if res is None else res.stride(0)
    thr, sc = drop_args(dropout)
    e.drop_thresh, e.drop_scale, e.seed = thr, sc, seed & 0xFFFFFFFFFFFFFFFF
    e.drop_ld = drop_ld if drop_ld is not None else N
    e.aux = ptr(aux)
    e.ldx = N if aux is None else aux.stride(0)
    e.aux_act = ACT[aux_act]
    e.post_scale = ptr(post_scale)
    e.colsum = ptr(colsum)
    e.colsum_accumulate = int(colsum_accumulate)
    if LAUNCH_PROBE is not None:
        LAUNCH_PROBE(d, e, lambda: check(lib().fer_gemm(C_ref(d), C_ref(e), stream()), "gemm"))
    else:
        check(lib().fer_gemm(C_ref(d), C_ref(e), stream()), "gemm")
    return out


def C_ref(x):
    import ctypes

    return ctypes.byref(x)


def linear_fwd(x, w, b=None, out=None, **kw):
    """y = x w^T + b for x [M,K], w [N,K] (nn.Linear)."""
    M, K = x.shape
    N = w.shape[0]
    if out is None:
        out = torch.empty(M, N, dtype=x.dtype, device=x.device)
    return gemm(x, w, out, M=M, N=N, K=K, bias=b, **kw)


def linear_dgrad(dy, w, out=None, **kw):
    """dx = dy w for dy [M,N], w [N,K]."""
    M, N = dy.shape
    K = w.shape[1]
    if out is None:
        out = torch.empty(M, K, dtype=dy.dtype, device=dy.device)
    return gemm(dy, w, out, a_kc=True, b_kc=False, M=M, N=K, K=N, lda=N, ldb=K, **kw)


def linear_wgrad_group(items, splits: int = 0):
    """dW_i (+)= dy_i^T x_i for several nn.Linear weights sharing the token count, in one launch
    (csrc/gemm.hip gemm_wgrad_group_kernel). items: (dy [M,N] bf16, x [M,K] bf16, out fp32 [N,K],
    accumulate) tuples; at most 8."""
    n = len(items)
    arr = (_lib.WgradItem * n)()
    for i, (dy, x, out, acc) in enumerate(items):
        _dev(dy)
        if dy.dtype != torch.bfloat16 or x.dtype != torch.bfloat16 or out.dtype != torch.float32:
            raise TypeError("linear_wgrad_group: bf16 dy / x and fp32 out")
        M, N = dy.shape
        K = x.shape[1]
        if x.shape[0] != M or tuple(out.shape) != (N, K) or dy.stride(1) != 1 or x.stride(1) != 1 or out.stride(1) != 1:
            raise ValueError("linear_wgrad_group: shapes / row-major layouts")
        arr[i] = _lib.WgradItem(dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0), out.data_ptr(), out.stride(0),
                                M, N, K, int(bool(acc)))
    nb = lib().fer_wgrad_group_ws(arr, n, splits)
    w = WS.get(nb, items[0][0].device, slot=1) if nb > 0 else None
    check(lib().fer_wgrad_group(arr, n, splits, ptr(w), 0 if w is None else w.numel() * 4, stream()), "wgrad_group")


def linear_wgrad(dy, x, out, accumulate=False, **kw):
    """dW (+)= dy^T x for dy [M,N], x [M,K]; out fp32 [N,K]."""
    M, N = dy.shape
    K = x.shape[1]
    return gemm(dy, x, out, a_kc=False, b_kc=False, M=N, N=K, K=M, lda=dy.stride(0), ldb=x.stride(0),
                accumulate=accumulate, **kw)


# ------------------------------------------------------------------ LayerNorm
def layernorm_fwd(x, w, b, eps, out=None, mean=None, rstd=None):
    M, D = x.shape
    out = torch.empty_like(x) if out is None else out
    check(lib().fer_layernorm_fwd(dcode(x), x.data_ptr(), x.stride(0), w.data_ptr(), b.data_ptr(), 1, 1,
                                  out.data_ptr(), out.stride(0), ptr(mean), ptr(rstd), M, D, eps, stream()),
          "layernorm_fwd")
    return out


def layernorm_bwd(dy, x, mean, rstd, w, dx=None, res=None, dx_drop=None, dropout=0.0, seed=0, dgamma=None,
                  dbeta=None, dbias=None, accumulate=False):
    M, D = x.shape
    dx = torch.empty_like(x) if dx is None else dx
    thr, sc = drop_args(dropout)
    nb = lib().fer_layernorm_bwd_ws(M, D)
    ws = WS.get(nb, x.device)
    check(lib().fer_layernorm_bwd(dcode(x), dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0), mean.data_ptr(),
                                  rstd.data_ptr(), w.data_ptr(), 1, 1, ptr(res), res.stride(0) if res is not None else D,
                                  dx.data_ptr(), dx.stride(0), ptr(dx_drop), thr, sc, seed & (2**64 - 1),
                                  ptr(dgamma), ptr(dbeta), ptr(dbias), int(accumulate), ws.data_ptr(), ws.numel() * 4,
                                  M, D, stream()), "layernorm_bwd")
    return dx


# ------------------------------------------------------------------ attention
def attention_saved(qkv, B, N, H, dh, dropout=0.0) -> torch.Tensor:
    """fp32 buffer for the state fer_attention_fwd keeps for the backward: lse [B*H*N] first
    (`saved[:B*H*N]`), then the dropout keep bits of the fast bf16 path."""
    thr, _ = drop_args(dropout)
    n = lib().fer_attention_saved_floats(dcode(qkv), B, N, H, dh, thr)
    return torch.empty(n, dtype=torch.float32, device=qkv.device)


def attention_fwd(qkv, out, saved, B, N, H, dh, dropout=0.0, seed=0):
    """out = attention(qkv); `saved` from attention_saved() (same B, N, H, dh, dropout)."""
    thr, sc = drop_args(dropout)
    nb = lib().fer_attention_ws(dcode(qkv), B, N, H)
    ws = WS.get(nb, qkv.device) if nb else None
    check(lib().fer_attention_fwd(dcode(qkv), qkv.data_ptr(), qkv.stride(0), out.data_ptr(), out.stride(0),
                                  saved.data_ptr(), saved.numel(), B, N, H, dh, 1.0 / math.sqrt(dh), thr, sc,
                                  seed & (2**64 - 1), ptr(ws), 0 if ws is None else ws.numel() * 4, stream()),
          "attention_fwd")
    return out


def attention_bwd(qkv, out, dout, saved, dqkv, B, N, H, dh, dropout=0.0, seed=0, colsum=None,
                  colsum_accumulate=False):
    """dqkv = d(attention)/d(qkv); colsum (fp32 [3*H*dh], optional) (+)= column sums of dqkv
    (the in_proj bias gradient), fused into the backward kernel."""
    thr, sc = drop_args(dropout)
    nb = lib().fer_attention_ws(dcode(qkv), B, N, H)
    ws = WS.get(nb, qkv.device) if nb else None
    check(lib().fer_attention_bwd(dcode(qkv), qkv.data_ptr(), qkv.stride(0), out.data_ptr(), out.stride(0),
                                  dout.data_ptr(), dout.stride(0), saved.data_ptr(), saved.numel(), dqkv.data_ptr(),
                                  dqkv.stride(0),
                                  ptr(ws), 0 if ws is None else ws.numel() * 4, B, N, H, dh, 1.0 / math.sqrt(dh),
                                  thr, sc, seed & (2**64 - 1), ptr(colsum), int(colsum_accumulate), stream()),
          "attention_bwd")
    return dqkv


# ------------------------------------------------------------------ misc
def colsum(x, out, accumulate=False, scale=None):
    M, N = x.shape
    ws = WS.get(lib().fer_colsum_ws(M, N), x.device)
    check(lib().fer_colsum(dcode(x), x.data_ptr(), x.stride(0), M, N, out.data_ptr(), int(accumulate), ptr(scale),
                           ws.data_ptr(), ws.numel() * 4, stream()), "colsum")
    return out


def im2col_patch(x, P, dtype):
    B, Cc, Hh, Ww = x.shape
    n = (Hh // P) * (Ww // P)
    K = Cc * P * P
    cols = torch.empty(B * n, K, dtype=dtype, device=x.device)
    check(lib().fer_im2col_patch(dcode(cols), x.data_ptr(), B, Cc, Hh, Ww, P, cols.data_ptr(), K, stream()),
          "im2col")
    return cols


def tokens_fwd(emb, cls, pos, B, n, D, dropout=0.0, seed=0):
    t = torch.empty(B * (n + 1), D, dtype=emb.dtype, device=emb.device)
    thr, sc = drop_args(dropout)
    check(lib().fer_tokens_fwd(dcode(emb), emb.data_ptr(), cls.data_ptr(), pos.data_ptr(), t.data_ptr(), B, n, D, thr,
                               sc, seed & (2**64 - 1), stream()), "tokens_fwd")
    return t


def tokens_bwd(dt, B, n, D, dcls, dpos, accumulate, dropout=0.0, seed=0, want_demb=True):
    demb = torch.empty(B * n, D, dtype=dt.dtype, device=dt.device) if want_demb else None
    thr, sc = drop_args(dropout)
    ws = WS.get(lib().fer_tokens_bwd_ws(B, n + 1, D), dt.device)
    check(lib().fer_tokens_bwd(dcode(dt), dt.data_ptr(), ptr(demb), ptr(dcls), ptr(dpos), int(accumulate), B, n, D,
                               thr, sc, seed & (2**64 - 1), ws.data_ptr(), ws.numel() * 4, stream()), "tokens_bwd")
    return demb


def head_fwd(t, N, lnw, lnb, eps, W, b, B, dropout=0.0, seed=0):
    D = t.shape[1]
    C = W.shape[0]
    logits = torch.empty(B, C, dtype=torch.float32, device=t.device)
    stats = torch.empty(B, 2, dtype=torch.float32, device=t.device)
    thr, sc = drop_args(dropout)
    check(lib().fer_head_fwd(dcode(t), t.data_ptr(), N * t.stride(0), lnw.data_ptr(), lnb.data_ptr(), eps,
                             W.data_ptr(), b.data_ptr(), logits.data_ptr(), stats.data_ptr(), B, D, C, thr, sc,
                             seed & (2**64 - 1), stream()), "head_fwd")
    return logits, stats


def head_bwd(t, N, lnw, lnb, W, stats, dlogits, B, grads, accumulate, dropout=0.0, seed=0):
    D = t.shape[1]
    C = W.shape[0]
    dt = torch.empty_like(t)
    thr, sc = drop_args(dropout)
    ws = WS.get(lib().fer_head_bwd_ws(B, D, C), t.device)
    g_lnw, g_lnb, g_W, g_b = grads
    check(lib().fer_head_bwd(dcode(t), t.data_ptr(), N * t.stride(0), lnw.data_ptr(), lnb.data_ptr(), W.data_ptr(),
                             stats.data_ptr(), dlogits.data_ptr(), dt.data_ptr(), 1, t.shape[0], t.stride(0),
                             ptr(g_lnw), ptr(g_lnb), ptr(g_W), ptr(g_b), int(accumulate), B, D, C, thr, sc,
                             seed & (2**64 - 1), ws.data_ptr(), ws.numel() * 4, stream()), "head_bwd")
    return dt


def cross_entropy(logits, labels, weight=None, label_smoothing=0.0, grad_scale=1.0, want_grad=True):
    B, Cc = logits.shape
    loss = torch.empty((), dtype=torch.float32, device=logits.device)
    dl = torch.empty_like(logits) if want_grad else None
    check(lib().fer_cross_entropy(logits.data_ptr(), labels.data_ptr(), ptr(weight), B, Cc, label_smoothing,
                                  grad_scale, loss.data_ptr(), ptr(dl), stream()), "cross_entropy")
    return loss, dl


def cast_bf16(x, out=None):
    out = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device) if out is None else out
    check(lib().fer_cast_f32_bf16(x.data_ptr(), out.data_ptr(), x.numel(), stream()), "cast")
    return out


def cast_f32(x, out=None):
    out = torch.empty(x.shape, dtype=torch.float32, device=x.device) if out is None else out
    check(lib().fer_cast_bf16_f32(x.data_ptr(), out.data_ptr(), x.numel(), stream()), "cast")
    return out


def axpy(x, t, scale_ptr, out=None):
    out = torch.empty_like(x) if out is None else out
    check(lib().fer_axpy(dcode(x), x.data_ptr(), t.data_ptr(), scale_ptr.data_ptr(), out.data_ptr(), x.numel(),
                         stream()), "axpy")
    return out


def dot(a, b, out, accumulate=False):
    ws = WS.get(4 * 1024 + 64, a.device, slot=2)
    check(lib().fer_dot(dcode(a), a.data_ptr(), ptr(b), a.numel(), out.data_ptr(), int(accumulate), ws.data_ptr(),
                        ws.numel() * 4, stream()), "dot")
    return out


def dropout(x, p, seed):
    out = torch.empty_like(x)
    thr, sc = drop_args(p)
    check(lib().fer_dropout(dcode(x), x.data_ptr(), out.data_ptr(), x.numel(), thr, sc, seed & (2**64 - 1), stream()),
          "dropout")
    return out
